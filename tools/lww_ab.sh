#!/bin/bash
# LWW write-pass shapes: sets.knobs 1 (half tiles, 512 threads) vs 17 (quarter tiles, 256 threads)
set -o pipefail
mkdir -p gpurun_out/lwab
timeout -k 10 300 python -u -m pytest tests/test_gpu_vclock_sets.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lwab/t.log 2>&1 || { tail -30 gpurun_out/lwab/t.log; exit 1; }
tail -1 gpurun_out/lwab/t.log
for k in 1 17 1 17; do
  timeout -k 10 200 python bench.py --workload lww_merge --no-cpu-baseline --option sets.knobs=$k > gpurun_out/lwab/b$k.json 2>gpurun_out/lwab/b.err || { tail -5 gpurun_out/lwab/b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/lwab/b$k.json')); print('knobs $k', d['ms_per_step'], d['roofline']['frac'])"
done
