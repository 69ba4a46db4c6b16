#!/bin/bash
# D2: tests + kernel stats, then A/B of the sort options, then the server-merge crossover.
bash tools/r03_d2.sh || exit $?
O=gpurun_out/d2ab; mkdir -p $O
for wl in lww_merge_d2 orset_merge_d2; do
  for opt in "sort.xcd_tiles=1" "sort.xcd_tiles=0" "sort.vec_up=0"; do
    timeout -k 10 120 python bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --option $opt > $O/$wl.$opt.json 2> $O/err || { tail -3 $O/err; exit 1; }
    echo "$wl $opt $(python -c "import json; d=json.load(open('$O/$wl.$opt.json')); print(d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])")"
  done
done
bash tools/r03_srv_cross.sh
