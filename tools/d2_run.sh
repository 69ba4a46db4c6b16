#!/bin/bash
# Fused D2 merge on the GPU box: parity tests, bench lines, rocprof stats.
set -o pipefail
O=gpurun_out/d2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_merge_unsorted.py tests/test_gpu_sort.py -x -v --timeout 120 \
  --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for wl in lww_merge_d2 orset_merge_d2; do
  timeout -k 10 180 python bench.py --workload $wl --steps 20 --warmup 3 > $O/b_$wl.json 2> $O/b_$wl.err || { cat $O/b_$wl.err; exit 1; }
  cat $O/b_$wl.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o d2 -- python3 $GRAFT_REPO_ROOT/bench.py --workload lww_merge_d2 --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
find $GRAFT_REPO_ROOT/$O/prof -name "*kernel_stats.csv" | head -3
