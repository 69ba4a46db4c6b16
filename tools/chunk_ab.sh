#!/bin/bash
# Set-merge schedule sweep on the GPU box: one bench line per (workload,
# option set).  Usage: tools/chunk_ab.sh "opt=v,opt=v" ["opt=v,..." ...]
set -o pipefail
O=gpurun_out/chunk_ab
mkdir -p $O
for wl in ${WLS:-lww_merge orset_merge}; do
  for cfg in "$@"; do
    args=""
    for o in ${cfg//,/ }; do args="$args --option $o"; done
    tag=$(echo "$cfg" | tr ',=' '_-')
    timeout -k 10 120 python bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline --no-e2e $args \
      > $O/b_${wl}_${tag}.json 2> $O/b_${wl}_${tag}.err || { echo "bench failed: $wl $cfg"; tail -5 $O/b_${wl}_${tag}.err; exit 1; }
    echo "$wl $cfg $(python -c "import json; d=json.load(open('$O/b_${wl}_${tag}.json')); print(d['ms_per_step'], d['roofline']['frac'])")"
  done
done
