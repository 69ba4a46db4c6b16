#!/bin/bash
# Server path after the ingest-validation rewrite: its tests, the ingest /
# merge phase split and two server_merge bench lines.
mkdir -p gpurun_out/srv3
timeout -k 10 300 python -u -m pytest tests/test_gpu_server_resident.py tests/test_gpu_server_errors.py tests/test_gpu_codec.py \
    tests/test_gossip_json.py -x -q --timeout 120 --timeout-method thread > gpurun_out/srv3/tests.log 2>&1 || { tail -30 gpurun_out/srv3/tests.log; exit 1; }
tail -1 gpurun_out/srv3/tests.log
CRDT_SRV_PROF=1 timeout -k 10 120 python -u tools/server_prof.py 5 > gpurun_out/srv3/prof5.txt 2> gpurun_out/srv3/prof5.err || exit 1
cat gpurun_out/srv3/prof5.txt; grep srv_ingest gpurun_out/srv3/prof5.err | tail -3; grep srv_merge gpurun_out/srv3/prof5.err | tail -2
for i in 1 2; do
timeout -k 10 200 python3 bench.py --workload server_merge --steps 50 --warmup 5 --no-e2e --cpu-seconds 3 > gpurun_out/srv3/bench$i.json || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/srv3/bench$i.json').read().strip().splitlines()[-1]); print('ms', d['ms_per_step'], 'M/s', round(d['value']/1e6,1), 'cpu M/s', round(d['cpu_baseline']['value']/1e6,1))"
done
