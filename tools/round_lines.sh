#!/bin/bash
# One bench line per workload (with its CPU baseline) into gpurun_out/round_bench/,
# and a summary line each: workload ms_per_step roofline.frac cpu_baseline.value.
O=gpurun_out/round_bench; mkdir -p $O
for wl in ${WLS:-shard_fold gcounter_join pncounter_join vclock_classify lww_merge orset_merge lww_merge_d2 orset_merge_d2 refmerge refmerge_delta gossip_round gossip_round_wire server_merge shard_set_merge loopback_set_merge loopback_orset_merge loopback_gossip_round}; do
  timeout -k 10 300 python bench.py --workload $wl --steps 20 --warmup 3 --cpu-seconds ${CPU_S:-4} > $O/$wl.json 2> $O/$wl.err || { echo "$wl failed"; tail -3 $O/$wl.err; exit 1; }
  echo "$wl $(python -c "import json; d=json.load(open('$O/$wl.json')); print(d['ms_per_step'], d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))")"
done
