#!/bin/bash
# Round-end check on the GPU box: GPU tests, smoke, and one bench line per workload.
set -o pipefail
O=gpurun_out/round
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for wl in ${WORKLOADS:-gcounter_join pncounter_join vclock_classify lww_merge orset_merge lww_merge_d2 orset_merge_d2 shard_fold refmerge refmerge_delta gossip_round}; do
  timeout -k 10 300 python bench.py --workload $wl > $O/bench_$wl.json 2> $O/bench_$wl.err || { tail -5 $O/bench_$wl.err; exit 1; }
  python -c "import json; d=json.load(open('$O/bench_$wl.json')); print('$wl', d['value'], d['unit'], d['ms_per_step'], d['roofline']['frac'])"
done
