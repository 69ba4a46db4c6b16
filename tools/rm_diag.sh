set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for d in 0 1 2; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/rmdiag$d -o run -- python3 $R/bench.py --workload refmerge --steps 10 --warmup 2 --no-cpu-baseline --option refmerge.diag_fold=$d > $R/gpurun_out/rmdiag$d.json
done
