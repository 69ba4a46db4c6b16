#!/bin/bash
mkdir -p gpurun_out/d2
timeout -k 10 400 python -u -m pytest tests/test_gpu_merge_unsorted.py tests/test_gpu_sort.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/d2/tests.log 2>&1
rc=$?; tail -3 gpurun_out/d2/tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/d2/tests.log | head -30; exit $rc; fi
bash tools/kstats.sh orset_merge_d2 && bash tools/kstats.sh gossip_round
