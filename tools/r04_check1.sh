#!/bin/bash
# Round-4 check: native population rounds, full-size configs[2] / D2 oracle
# tests, gossip / local-apply suites, shard_set_merge N=1 bench line.
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_population.py tests/test_gpu_gossip.py \
    tests/test_gpu_local_apply.py tests/test_gpu_full_configs.py -m gpu -x -v --timeout 400 \
    --timeout-method thread > gpurun_out/r4_check1.log 2>&1
rc=$?
tail -15 gpurun_out/r4_check1.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --workload shard_set_merge --steps 20 --warmup 3 --no-cpu-baseline --no-e2e \
    > gpurun_out/r4_shard_set_merge.json 2> gpurun_out/r4_shard_set_merge.err || exit $?
timeout -k 10 300 python -u bench.py --workload lww_merge --steps 20 --warmup 3 --no-cpu-baseline --no-e2e \
    > gpurun_out/r4_lww_merge.json 2> gpurun_out/r4_lww_merge.err || exit $?
python3 -c "
import json
for w in ('shard_set_merge','lww_merge'):
    d=json.loads(open('gpurun_out/r4_%s.json'%w).read())
    print(w, d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])
"
