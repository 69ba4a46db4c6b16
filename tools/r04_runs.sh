#!/bin/bash
# Sampled D2 plans from 256 runs of 64 consecutive tuples per side (new)
# against 32768 strided single tuples (crdt_amd/ab_base): D2 parity (incl.
# the redo path), then alternating bench lines of both D2 merges.
set -o pipefail
OUT=gpurun_out/runs; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_merge_unsorted.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 bash tools/ab_build.sh lww_merge_d2 3 || exit 1
timeout -k 10 600 bash tools/ab_build.sh orset_merge_d2 2 || exit 1
