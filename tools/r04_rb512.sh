#!/bin/bash
# OR-Set D2 dedup workgroups of 1024 threads (3 elements each) against 512 (6):
# parity, then alternating bench lines against crdt_amd/ab_base (RB = 512, in-tree RB = 1024).
set -o pipefail
OUT=gpurun_out/rb512; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_merge_unsorted.py tests/test_gpu_sort.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 bash tools/ab_build.sh orset_merge_d2 3
