#!/bin/bash
# Gossip round (1000 x 10k, population rounds): the kv tile pass as two
# launches (one-pair tiles, the rest) vs one launch holding both paths.
mkdir -p gpurun_out/kvx
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in 0 1 0 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kvx/t$v -o run -- \
      python3 $R/bench.py --workload gossip_round --steps 20 --warmup 3 --no-e2e --no-cpu-baseline --option refmerge.kv_one_launch=$v \
      > $R/gpurun_out/kvx/b$v.json 2> $R/gpurun_out/kvx/b$v.err || { tail -3 $R/gpurun_out/kvx/b$v.err; exit 1; }
  python3 - $R/gpurun_out/kvx/t$v/run_kernel_stats.csv $R/gpurun_out/kvx/b$v.json $v <<'PY'
import csv, json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print("kv_one_launch", sys.argv[3], "ms/step", d["ms_per_step"], "frac", d["roofline"]["frac"])
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_rm_tile' in r['Name']:
        print("   ", f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:50]}")
PY
done
