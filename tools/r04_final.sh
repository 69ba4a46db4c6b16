#!/bin/bash
# Round-4 closing evidence on one MI355X: the whole -m gpu suite, smoke(),
# the default bench line (configs[4] E1 shard_fold) with its rocprofv3 stats
# and FETCH / WRITE PMC passes (tools/profile.sh), and the server_merge line.
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/final/gpu_tests.log 2>&1 || { tail -40 gpurun_out/final/gpu_tests.log; exit 1; }
tail -2 gpurun_out/final/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" \
    > gpurun_out/final/smoke.log 2>&1 || { tail -20 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/final/bench_default.json 2> gpurun_out/final/bench_default.err || { tail gpurun_out/final/bench_default.err; exit 1; }
cat gpurun_out/final/bench_default.json
timeout -k 10 300 python bench.py --workload server_merge --steps 50 --warmup 5 --no-e2e --cpu-seconds 3 \
    > gpurun_out/final/bench_server_merge.json 2> gpurun_out/final/bench_server_merge.err || exit 1
timeout -k 10 700 bash tools/profile.sh shard_fold || exit 1
CRDT_SRV_PROF=1 timeout -k 10 120 python -u tools/server_prof.py 5 > gpurun_out/final/srv_prof5.txt 2> gpurun_out/final/srv_prof5.err || exit 1
grep srv_ingest gpurun_out/final/srv_prof5.err | tail -5; tail -2 gpurun_out/final/srv_prof5.err
timeout -k 10 200 python bench.py --workload gossip_round_wire --steps 10 --warmup 2 --no-e2e --no-cpu-baseline > gpurun_out/final/bench_wire.json 2> gpurun_out/final/bench_wire.err || exit 1
timeout -k 10 600 bash tools/server_cross.sh > gpurun_out/final/server_cross.txt 2>&1 || exit 1
cat gpurun_out/final/server_cross.txt
