#!/bin/bash
# Server.merge() after the pinned staging / ingest-time upload / incremental
# CurrentState changes: its parity tests, the phase split and the kernel list.
mkdir -p gpurun_out/srv2
timeout -k 10 500 python -u -m pytest tests/test_gpu_server_resident.py tests/test_gpu_server_errors.py tests/test_gpu_codec.py \
    tests/test_gpu_gossip.py tests/test_gpu_population.py tests/test_gpu_refmerge.py tests/test_gpu_refmerge_edges.py tests/test_gpu_replay_delta.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/srv2/tests.log 2>&1 || { tail -30 gpurun_out/srv2/tests.log; exit 1; }
tail -2 gpurun_out/srv2/tests.log
CRDT_SRV_PROF=1 timeout -k 10 120 python -u tools/server_prof.py 5 > gpurun_out/srv2/prof5.txt 2> gpurun_out/srv2/prof5.err || { tail gpurun_out/srv2/prof5.err; exit 1; }
cat gpurun_out/srv2/prof5.txt; tail -4 gpurun_out/srv2/prof5.err
for i in 1 2; do
timeout -k 10 200 python3 bench.py --workload server_merge --steps 50 --warmup 5 --no-e2e --cpu-seconds 3 > gpurun_out/srv2/bench$i.json || exit 1
python3 -c "import json,sys; d=json.loads(open('gpurun_out/srv2/bench$i.json').read().strip().splitlines()[-1]); print('ms', d['ms_per_step'], 'M/s', d['value']/1e6, 'cpu M/s', d['cpu_baseline']['value']/1e6)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/srv2/trace -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --workload server_merge --steps 20 --warmup 3 --no-e2e --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/srv2/bench_prof.json || exit 1
