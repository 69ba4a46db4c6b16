#!/bin/bash
# A/B of two builds in one GPU call: crdt_amd/ab_base/libcrdt_amd.so (baseline, copied before the
# change) against the in-tree build.  TESTS: parity files run on the in-tree build first.
#   TESTS="..." WLS="..." tools/ab2.sh
set -o pipefail
O=gpurun_out/ab2
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
    || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for rep in 1 2 3; do
for wl in $WLS; do
  for b in base new; do
    if [ $b = base ]; then export CRDT_AMD_LIB=$PWD/crdt_amd/ab_base/libcrdt_amd.so; else unset CRDT_AMD_LIB; fi
    timeout -k 10 120 python bench.py --workload $wl --steps 30 --warmup 3 --no-cpu-baseline > $O/b_${wl}_$b.json 2> $O/b_${wl}_$b.err || { tail -5 $O/b_${wl}_$b.err; exit 1; }
    echo "$wl $b $(python -c "import json; d=json.load(open('$O/b_${wl}_$b.json')); print(d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])")"
  done
done
done
unset CRDT_AMD_LIB
