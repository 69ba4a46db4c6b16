#!/bin/bash
# OR count-pass staging A/B + the new two-stream test
O=gpurun_out/b3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_counters.py tests/test_gpu_vclock_sets.py -m gpu -q \
  --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $O/tests.log | head -30; exit $rc; fi
for o in sets.or_count_dma=0 sets.or_count_dma=1 sets.or_count_dma=0 sets.or_count_dma=1; do
  timeout -k 10 120 python bench.py --workload orset_merge --steps 30 --warmup 3 --no-cpu-baseline --no-e2e --option $o > $O/or_$o.json 2> $O/or_$o.err || exit 1
  echo "orset_merge $o $(python -c "import json; d=json.load(open('$O/or_$o.json')); print(d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])")"
done
