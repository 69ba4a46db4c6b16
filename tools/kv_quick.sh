mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_gossip.py tests/test_gpu_refmerge.py > gpurun_out/kvq.log 2>&1 || { tail -30 gpurun_out/kvq.log; exit 1; }
tail -1 gpurun_out/kvq.log
CRDT_GOSSIP_PULL=inplace timeout -k 10 200 python bench.py --workload gossip_round --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/kvq_inplace.json 2>/dev/null && python -c "import json; d=json.load(open('gpurun_out/kvq_inplace.json')); print('inplace', d['ms_per_step'], d['roofline']['frac'])"
