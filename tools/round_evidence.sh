#!/bin/bash
# Round evidence: GPU suite + default bench (tools/gpu_suite.sh), smoke, then rocprofv3 stats + FETCH/WRITE PMC
# per workload (tools/profile.sh), then one bench line per workload with the CPU baseline.
bash tools/gpu_suite.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
WLS="shard_fold lww_merge orset_merge lww_merge_d2 orset_merge_d2 refmerge refmerge_delta gossip_round" bash tools/profiles_all.sh || exit $?
O=gpurun_out/round_bench; mkdir -p $O
for wl in lww_merge orset_merge lww_merge_d2 orset_merge_d2 refmerge refmerge_delta gossip_round gossip_round_wire server_merge shard_set_merge; do
  timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 3 > $O/$wl.json 2> $O/$wl.err || { echo "$wl failed"; tail -3 $O/$wl.err; exit 1; }
  echo "$wl $(python -c "import json; d=json.load(open('$O/$wl.json')); print(d['ms_per_step'], d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))")"
done
