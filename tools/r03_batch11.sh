#!/bin/bash
# gossip rounds with one read-back per round: their GPU tests, then the bench lines
mkdir -p gpurun_out/gos
timeout -k 10 600 python -u -m pytest tests/test_gpu_gossip.py tests/test_gpu_multirank.py tests/test_gpu_seg.py tests/test_gpu_codec.py tests/test_gpu_shard_sets.py tests/test_gpu_shard_refmerge.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/gos/tests.log 2>&1
rc=$?; tail -3 gpurun_out/gos/tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/gos/tests.log | head -30; exit $rc; fi
for wl in gossip_round gossip_round_wire; do
  timeout -k 10 200 python bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/gos/$wl.json 2> gpurun_out/gos/$wl.err || { tail -3 gpurun_out/gos/$wl.err; exit 1; }
  echo "$wl $(python -c "import json; d=json.load(open('gpurun_out/gos/$wl.json')); print(d['ms_per_step'], d['roofline']['frac'])")"
done
