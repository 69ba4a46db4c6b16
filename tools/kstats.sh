#!/bin/bash
# rocprofv3 --kernel-trace --stats of one bench workload (no counters): per-kernel averages.
# Usage: [KS_TAG=_x] tools/kstats.sh <workload> [extra bench args...]
wl=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/ks_${wl}${KS_TAG}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline --no-e2e "$@" > $O/bench.json 2> $O/bench.err || exit 1
python3 - "$O/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    if any(x in n for x in ("stream_", "synth", "elementwise", "rocclr")): continue
    print(f"  {n[:64]:64s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:9.1f}")
PY
