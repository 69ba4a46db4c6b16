#!/bin/bash
# OR-Set D2 key-bucket counting sorts (sort.or_table): the D2 / sort / full
# config suites, then A/B pairs of the orset_merge_d2 bench line (tables on /
# off) under rocprofv3 --stats in one call.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ortab
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_merge_unsorted.py tests/test_gpu_sort.py tests/test_gpu_full_configs.py -m gpu -x -v \
    --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
cd /tmp && export TMPDIR=/tmp
for v in 1 0 1 0; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t_$v -o run -- \
      python3 $R/bench.py --workload orset_merge_d2 --steps 20 --warmup 3 --no-e2e --no-cpu-baseline --option sort.or_table=$v \
      > $OUT/b_$v.json 2> $OUT/b_$v.err || { tail -3 $OUT/b_$v.err; exit 1; }
  python3 - $OUT/t_$v/run_kernel_stats.csv $OUT/b_$v.json "or_table=$v" <<'PY'
import csv, json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[3], "ms/step", d["ms_per_step"], "frac", d["roofline"]["frac"])
for r in csv.DictReader(open(sys.argv[1])):
    if 'crdt' in r['Name']:
        print("   ", f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:60]}")
PY
done
