#!/bin/bash
# Fused kv output of the merge (crdt_refmerge_batch_kv): its parity tests and
# the gossip / server suites, then the gossip bench lines and kernel stats.
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_refmerge.py tests/test_gpu_gossip.py tests/test_gpu_server_resident.py tests/test_gpu_server_errors.py tests/test_gpu_codec.py tests/test_gpu_refmerge_edges.py \
  > gpurun_out/kv_tests.log 2>&1 || { tail -30 gpurun_out/kv_tests.log; exit 1; }
tail -2 gpurun_out/kv_tests.log
for wl in gossip_round gossip_round_wire; do
  timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/kv_$wl.json 2> gpurun_out/kv_$wl.err || { tail -5 gpurun_out/kv_$wl.err; exit 1; }
  echo "$wl $(python -c "import json; d=json.load(open('gpurun_out/kv_$wl.json')); print(d['ms_per_step'], d['roofline']['frac'])")"
done
bash tools/kstats.sh gossip_round
CRDT_GOSSIP_PULL=inplace timeout -k 10 300 python bench.py --workload gossip_round --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/kv_gossip_inplace.json 2>/dev/null && python -c "import json; d=json.load(open('gpurun_out/kv_gossip_inplace.json')); print('inplace', d['ms_per_step'], d['roofline']['frac'])"
