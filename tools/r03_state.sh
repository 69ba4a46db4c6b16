#!/bin/bash
# State check: GPU suite + default bench, then one bench line per main workload.
bash tools/gpu_suite.sh || exit $?
O=gpurun_out/state; mkdir -p $O
for wl in lww_merge orset_merge lww_merge_d2 orset_merge_d2 refmerge refmerge_delta gossip_round server_merge; do
  timeout -k 10 200 python bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline > $O/$wl.json 2> $O/$wl.err || { echo "$wl failed"; tail -3 $O/$wl.err; exit 1; }
  echo "$wl $(python -c "import json; d=json.load(open('$O/$wl.json')); print(d['ms_per_step'], d['roofline'].get('avg_launch_us'), d['roofline']['frac'], d.get('value'))")"
done
