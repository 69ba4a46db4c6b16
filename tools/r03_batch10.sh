#!/bin/bash
mkdir -p gpurun_out/d2
timeout -k 10 400 python -u -m pytest tests/test_gpu_merge_unsorted.py tests/test_gpu_sort.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/d2/tests.log 2>&1
rc=$?; tail -3 gpurun_out/d2/tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/d2/tests.log | head -30; exit $rc; fi
bash tools/kstats.sh orset_merge_d2 | grep -E "rdd|pass|minmax|up" && \
for m in 2 1; do timeout -k 10 120 python bench.py --workload orset_merge_d2 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --option sort.or_key_only=$m > gpurun_out/d2/m$m.json 2>/dev/null && echo "or_key_only=$m $(python -c "import json; d=json.load(open('gpurun_out/d2/m$m.json')); print(d['ms_per_step'], d['roofline']['frac'])")"; done
