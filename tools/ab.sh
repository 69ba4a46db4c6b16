#!/bin/bash
# Generic A/B on the GPU box.
#   TESTS="<pytest files>" TOPT="<CRDT_TEST_OPTIONS variant>" WLS="<workloads>" tools/ab.sh opt1 opt2 ...
# parity (default knobs, then TOPT), then two rounds of bench lines per (workload, option).
set -o pipefail
O=gpurun_out/ab
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 \
    || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
  if [ -n "$TOPT" ]; then
    CRDT_TEST_OPTIONS="$TOPT" timeout -k 10 400 python -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread \
      > $O/tests_opt.log 2>&1 || { echo "opt tests failed"; tail -30 $O/tests_opt.log; exit 1; }
    tail -1 $O/tests_opt.log
  fi
fi
for rep in 1 2; do
for wl in $WLS; do
  for v in "$@"; do
    timeout -k 10 120 python bench.py --workload $wl --steps 30 --warmup 3 --no-cpu-baseline --option $v > $O/b_${wl}_$v.json 2> $O/b_${wl}_$v.err || { tail -5 $O/b_${wl}_$v.err; exit 1; }
    echo "$wl $v $(python -c "import json; d=json.load(open('$O/b_${wl}_$v.json')); print(d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])")"
  done
done
done
