#!/bin/bash
# RefMerge tile pass per workgroup shape (refmerge.tile_parts), after the RefMerge suites
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_refmerge.py tests/test_gpu_vclock_sets.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rmp_t.log 2>&1 || { tail -30 gpurun_out/rmp_t.log; exit 1; }
tail -1 gpurun_out/rmp_t.log
for r in a b; do for p in 1 2 4; do
  bash tools/kstats.sh r$p$r refmerge --option refmerge.tile_parts=$p | grep k_rm_tile
done; done
