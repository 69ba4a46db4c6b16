#!/bin/bash
O=gpurun_out/b4; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_merge_unsorted.py tests/test_gpu_sort.py -m gpu -q \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $O/tests.log | head -30; exit $rc; fi
for wl in lww_merge_d2 orset_merge_d2; do
  timeout -k 10 200 python bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/$wl.json 2> $O/$wl.err || exit 1
  echo "$wl $(python -c "import json; d=json.load(open('$O/$wl.json')); print(d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])")"
done
bash tools/ab_build.sh lww_merge 2 && bash tools/ab_build.sh orset_merge 2
