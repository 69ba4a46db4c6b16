#!/bin/bash
# A/B of the in-tree library against another build (crdt_amd/ab_base/libcrdt_amd.so,
# e.g. an earlier commit's csrc built with make LIB=...): alternating bench lines.
# Usage: tools/ab_build.sh <workload> [reps] [extra bench args...]
wl=$1; reps=${2:-2}; shift 2
O=gpurun_out/ab_$wl; mkdir -p $O
for r in $(seq $reps); do
  for b in base new; do
    if [ $b = base ]; then export CRDT_AMD_LIB=$PWD/crdt_amd/ab_base/libcrdt_amd.so; else unset CRDT_AMD_LIB; fi
    timeout -k 10 150 python bench.py --workload $wl --steps 30 --warmup 3 --no-cpu-baseline --no-e2e "$@" > $O/$b$r.json 2> $O/$b$r.err || { tail -3 $O/$b$r.err; exit 1; }
    echo "$wl $b $(python -c "import json; d=json.load(open('$O/$b$r.json')); print(d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])")"
  done
done
