#!/bin/bash
# Per-kernel rocprofv3 stats of a bench workload under bench options: tools/kstats.sh <tag> <workload> [bench args]
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; tag=$1; wl=$2; shift 2
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ks_$tag -o run -- \
  python3 $R/bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-e2e "$@" > $R/gpurun_out/ks_$tag.json
python3 - $R/gpurun_out/ks_$tag/run_kernel_stats.csv $tag <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for x in rows:
    if int(x['Calls']) >= 10:
        print(sys.argv[2], x['Name'][:48], x['Calls'], round(float(x['AverageNs']) / 1e3, 1))
PY
