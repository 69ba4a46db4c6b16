#!/bin/bash
mkdir -p gpurun_out/b14
timeout -k 10 600 python -u -m pytest tests/test_gpu_merge_unsorted.py tests/test_gpu_sort.py tests/test_gpu_gossip.py tests/test_gpu_multirank.py tests/test_gpu_shard_sets.py tests/test_gpu_shard_refmerge.py -m gpu -x -q \
  --timeout 300 --timeout-method thread > gpurun_out/b14/tests.log 2>&1
rc=$?; tail -3 gpurun_out/b14/tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/b14/tests.log | head -30; exit $rc; fi
for wl in lww_merge_d2 orset_merge_d2 gossip_round gossip_round_wire; do
  timeout -k 10 200 python bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/b14/$wl.json 2> gpurun_out/b14/$wl.err || { tail -3 gpurun_out/b14/$wl.err; exit 1; }
  echo "$wl $(python -c "import json; d=json.load(open('gpurun_out/b14/$wl.json')); print(d['ms_per_step'], d['roofline']['frac'])")"
done
bash tools/kstats.sh lww_merge_d2 | grep -E "dd_"
