#!/bin/bash
# A/B of set-merge variants on the GPU box: parity tests, bench lines per option.
# Usage: tools/set_ab.sh "opt=v" ["opt=v" ...]
set -o pipefail
O=gpurun_out/set_ab
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_vclock_sets.py tests/test_gpu_shard_sets.py tests/test_gpu_sort.py \
  -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for wl in lww_merge orset_merge; do
  for opt in "$@"; do
    timeout -k 10 120 python bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline --option $opt > $O/b_${wl}_${opt}.json 2> $O/b_${wl}_${opt}.err || exit 1
    echo "$wl $opt $(python -c "import json,sys; d=json.load(open('$O/b_${wl}_${opt}.json')); print(d['ms_per_step'], d['roofline']['frac'])")"
  done
done
