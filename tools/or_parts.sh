#!/bin/bash
# OR-Set write pass per workgroup shape (sets.or_parts), after the set suite
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_vclock_sets.py -x -q --timeout 120 --timeout-method thread > gpurun_out/orp_t.log 2>&1 || { tail -30 gpurun_out/orp_t.log; exit 1; }
tail -1 gpurun_out/orp_t.log
for r in a b; do for p in 1 2 4; do
  bash tools/kstats.sh o$p$r orset_merge --option sets.or_parts=$p | grep k_or_write
done; done
