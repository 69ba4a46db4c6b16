#!/bin/bash
# Wire rounds on one-pair populations (the decode counts multi-pair entries):
# parity, then the wire round and server_merge lines.
mkdir -p gpurun_out/wire1p
timeout -k 10 400 python -u -m pytest tests/test_gpu_population.py tests/test_gpu_codec.py tests/test_gpu_server_resident.py \
    tests/test_gpu_gossip.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/wire1p/tests.log 2>&1 \
    || { tail -30 gpurun_out/wire1p/tests.log; exit 1; }
tail -1 gpurun_out/wire1p/tests.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --workload gossip_round_wire --steps 10 --warmup 2 --no-e2e --no-cpu-baseline > gpurun_out/wire1p/w$i.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/wire1p/w$i.json').read().strip().splitlines()[-1]); print('wire', d['ms_per_step'], d['roofline']['frac'])"
done
timeout -k 10 200 python bench.py --workload server_merge --steps 50 --warmup 5 --no-e2e --cpu-seconds 2 > gpurun_out/wire1p/srv.json 2>/dev/null || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/wire1p/srv.json').read().strip().splitlines()[-1]); print('server_merge', d['ms_per_step'], d['value']/1e6, d['cpu_baseline']['value']/1e6)"
