#!/bin/bash
# OR-Set D2: groups of <= 8 tuples resolved in registers (new) against the
# LDS walks (crdt_amd/ab_base); sort.or_key_only 2 (key + 9 tag bits, 4
# passes) and 3 (key + 1 tag bit, 3 passes).
set -o pipefail
OUT=gpurun_out/orreg; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_merge_unsorted.py tests/test_gpu_sort.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 1 2; do
  for v in base:2 new:2 new:3; do
    b=${v%%:*}; m=${v##*:}
    if [ $b = base ]; then export CRDT_AMD_LIB=$PWD/crdt_amd/ab_base/libcrdt_amd.so; else unset CRDT_AMD_LIB; fi
    timeout -k 10 150 python bench.py --workload orset_merge_d2 --steps 30 --warmup 3 --no-cpu-baseline --no-e2e \
        --option sort.or_key_only=$m > $OUT/${b}_${m}_$r.json 2> $OUT/${b}_${m}_$r.err || { tail -3 $OUT/${b}_${m}_$r.err; exit 1; }
    echo "$b mode=$m $(python -c "import json; d=json.load(open('$OUT/${b}_${m}_$r.json')); print(d['ms_per_step'], d['roofline']['frac'])")"
  done
done
unset CRDT_AMD_LIB
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t3 -o run -- \
    python3 bench.py --workload orset_merge_d2 --steps 20 --warmup 3 --no-e2e --no-cpu-baseline --option sort.or_key_only=3 > $OUT/t3.json 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t2 -o run -- \
    python3 bench.py --workload orset_merge_d2 --steps 20 --warmup 3 --no-e2e --no-cpu-baseline --option sort.or_key_only=2 > $OUT/t2.json 2>&1 || exit 1
for m in 2 3; do echo "mode $m"; python3 -c "
import csv
for r in csv.DictReader(open('$OUT/t$m/run_kernel_stats.csv')):
    if 'crdt' in r['Name']: print('   ', f\"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:60]}\")
"; done
