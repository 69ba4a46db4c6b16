#!/bin/bash
# LWW write pass per workgroup shape (sets.lww_parts), after the set suite
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_vclock_sets.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lwp_t.log 2>&1 || { tail -30 gpurun_out/lwp_t.log; exit 1; }
tail -1 gpurun_out/lwp_t.log
for r in a b; do for p in 2 4 8 16; do
  bash tools/kstats.sh p$p$r lww_merge --option sets.lww_parts=$p | grep k_lww_write
done; done
