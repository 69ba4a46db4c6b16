#!/bin/bash
# OR-Set D2 key chunks sorted in LDS (two radix passes on the top 16 key bits):
# D2 parity, then on / off pairs of the bench line.

set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/ortab2
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_merge_unsorted.py tests/test_gpu_sort.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
cd /tmp && export TMPDIR=/tmp
for v in lb1 lb0 lb1 lb0; do
  case $v in lb?) opt="--option sort.or_lookback=${v#lb}";; d?) opt="--option sort.rdd_diag=${v#d}";; on) opt="--option sort.or_table=1";; off) opt="--option sort.or_table=0";; esac
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t_$v -o run -- \
      python3 $R/bench.py --workload orset_merge_d2 --steps 20 --warmup 3 --no-e2e --no-cpu-baseline $opt \
      > $OUT/b_$v.json 2> $OUT/b_$v.err || { tail -3 $OUT/b_$v.err; exit 1; }
  python3 - $OUT/t_$v/run_kernel_stats.csv $OUT/b_$v.json "$v" <<'PY'
import csv, json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ks = {r['Name'][:40]: float(r['AverageNs'])/1e3 for r in csv.DictReader(open(sys.argv[1])) if 'crdt' in r['Name']}
print(sys.argv[3], "ms/step", d["ms_per_step"], " ".join(f"{k.split('(')[0].split('::')[-1]}={v:.1f}" for k, v in ks.items() if 'synth' not in k))
PY
done
