#!/bin/bash
# Composing upsweep keeping only the digits in registers (31 VGPRs, 8 waves
# per SIMD, against 79 / 6): D2 / sort parity, then alternating bench lines
# of both D2 merges against crdt_amd/ab_base.
set -o pipefail
OUT=gpurun_out/upv; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_merge_unsorted.py tests/test_gpu_sort.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 bash tools/ab_build.sh lww_merge_d2 3 || exit 1
timeout -k 10 600 bash tools/ab_build.sh orset_merge_d2 2 || exit 1
