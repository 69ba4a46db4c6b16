#!/bin/bash
# LWW D2 tables, second step: plan read-back through pinned memory, and the
# minmax grid (sort.mm_blocks_per_cu 1 / 2 / 4) under the table path.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/lwwtab2
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_merge_unsorted.py tests/test_gpu_sort.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
cd /tmp && export TMPDIR=/tmp
run() {  # tag workload options...
  tag=$1; wl=$2; shift 2
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t_$tag -o run -- \
      python3 $R/bench.py --workload $wl --steps 20 --warmup 3 --no-e2e --no-cpu-baseline "$@" \
      > $OUT/b_$tag.json 2> $OUT/b_$tag.err || { tail -3 $OUT/b_$tag.err; exit 1; }
  python3 - $OUT/t_$tag/run_kernel_stats.csv $OUT/b_$tag.json "$tag" <<'PY'
import csv, json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[3], "ms/step", d["ms_per_step"], "frac", d["roofline"]["frac"])
for r in csv.DictReader(open(sys.argv[1])):
    if r['Name'].startswith('crdt::') or r['Name'].startswith('void crdt::k_sort') or 'k_lww_table' in r['Name'] or 'k_dd' in r['Name']:
        print("   ", f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:60]}")
PY
}
for rep in 1 2; do
  for m in 1 2 4; do run lww_mm${m}_$rep lww_merge_d2 --option sort.mm_blocks_per_cu=$m; done
done

run or_3 orset_merge_d2 --option sort.or_key_only=3
run or_2b orset_merge_d2
run or_3b orset_merge_d2 --option sort.or_key_only=3
