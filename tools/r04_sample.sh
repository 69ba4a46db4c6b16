#!/bin/bash
# D2 dense-key paths from a sampled plan (sort.sample_plan): D2 / sort /
# full-config parity, then A/B pairs of both D2 bench lines in one call.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/sample
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_merge_unsorted.py tests/test_gpu_sort.py tests/test_gpu_full_configs.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
cd /tmp && export TMPDIR=/tmp
for wl in lww_merge_d2 orset_merge_d2; do
for v in 1 0 1 0; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/t_${wl}_$v -o run -- \
      python3 $R/bench.py --workload $wl --steps 20 --warmup 3 --no-e2e --no-cpu-baseline --option sort.sample_plan=$v \
      > $OUT/b_${wl}_$v.json 2> $OUT/b_${wl}_$v.err || { tail -3 $OUT/b_${wl}_$v.err; exit 1; }
  python3 - $OUT/t_${wl}_$v/run_kernel_stats.csv $OUT/b_${wl}_$v.json "$wl sample=$v" <<'PY'
import csv, json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
ks = {r['Name'][:40]: float(r['AverageNs'])/1e3 for r in csv.DictReader(open(sys.argv[1])) if 'crdt' in r['Name'] and 'synth' not in r['Name'] and 'stream' not in r['Name']}
print(sys.argv[3], "ms/step", d["ms_per_step"], " ".join(f"{k.split('(')[0].split('::')[-1]}={v:.1f}" for k, v in ks.items()))
PY
done
done
