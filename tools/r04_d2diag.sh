#!/bin/bash
# Where the D2 LWW dedup apply's time goes: sort.rdd_diag 0 (full), 1 (load +
# LDS only), 2 (+ emit flags and ranks, no stores); kernel stats per run.
mkdir -p gpurun_out/d2diag
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for d in 0 1 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/d2diag/t$d -o run -- \
      python3 $R/bench.py --workload lww_merge_d2 --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --option sort.rdd_diag=$d \
      > $R/gpurun_out/d2diag/b$d.json 2> $R/gpurun_out/d2diag/b$d.err || { tail -3 $R/gpurun_out/d2diag/b$d.err; exit 1; }
  python3 - $R/gpurun_out/d2diag/t$d/run_kernel_stats.csv $d <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_dd_' in r['Name'] or 'k_sort' in r['Name']:
        print(sys.argv[2], f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:70]}")
PY
done
