#!/bin/bash
# Round-4 closing run (final tree): the whole -m gpu suite, smoke(),
# the default bench line and the bench lines (with CPU baselines) of the
# workloads this round changed.
mkdir -p gpurun_out/final8
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/final8/gpu_tests.log 2>&1 || { tail -40 gpurun_out/final8/gpu_tests.log; exit 1; }
tail -1 gpurun_out/final8/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('__SMOKE_OK__')" \
    > gpurun_out/final8/smoke.log 2>&1 || { tail -20 gpurun_out/final8/smoke.log; exit 1; }
tail -1 gpurun_out/final8/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/final8/bench_default.json 2> gpurun_out/final8/bench_default.err || { tail gpurun_out/final8/bench_default.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/final8/bench_default.json').read().strip().splitlines()[-1]); print('default', d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'])"
for wl in server_merge gossip_round gossip_round_wire refmerge lww_merge orset_merge lww_merge_d2 orset_merge_d2; do
  timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 3 > gpurun_out/final8/$wl.json 2> gpurun_out/final8/$wl.err || { echo "$wl failed"; tail -3 gpurun_out/final8/$wl.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/final8/$wl.json').read().strip().splitlines()[-1]); c=d.get('cpu_baseline') or {}; print('$wl', d['ms_per_step'], d['roofline']['frac'], d['value'], c.get('value'))"
done
