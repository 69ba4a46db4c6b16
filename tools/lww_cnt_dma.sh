#!/bin/bash
# LWW count pass staged by LDS-DMA (default) against register staging (sets.knobs bit 3)
set -o pipefail
CRDT_TEST_OPTIONS="sets.knobs=9" timeout -k 10 300 python -u -m pytest tests/test_gpu_vclock_sets.py tests/test_gpu_shard_sets.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lcd_t.log 2>&1 || { tail -30 gpurun_out/lcd_t.log; exit 1; }
tail -1 gpurun_out/lcd_t.log
for r in a b c; do for k in 1 9; do
  bash tools/kstats.sh lcd$k$r lww_merge --option sets.knobs=$k | grep k_lww_count | sed "s/^/k$k /"
  python -c "import json; d=json.load(open('gpurun_out/ks_lcd$k$r.json')); print('knobs $k', d['ms_per_step'])"
done; done
