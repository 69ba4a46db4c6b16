# RefMerge knob sweep: bench refmerge per knob setting (rocprof kernel stats each)
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for kv in "$@"; do
  tag=$(echo $kv | tr '=,.' '___')
  opts=""; for o in $(echo $kv | tr ',' ' '); do opts="$opts --option $o"; done
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/rmk_$tag -o run -- python3 $R/bench.py --workload refmerge --steps 10 --warmup 2 --no-cpu-baseline $opts > $R/gpurun_out/rmk_$tag.json
done
