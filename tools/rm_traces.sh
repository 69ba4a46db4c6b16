# rocprofv3 kernel stats of bench workloads: tools/rm_traces.sh tag "workload[:opt=v,...]" ...
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
tag=$1; shift
for spec in "$@"; do
  wl=${spec%%:*}; opts=""
  if [ "$wl" != "$spec" ]; then for o in $(echo ${spec#*:} | tr ',' ' '); do opts="$opts --option $o"; done; fi
  name=$(echo $spec | tr ':=,.' '____')
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$tag/$name -o run -- python3 $R/bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline $opts > $R/gpurun_out/$tag/$name.json
done
