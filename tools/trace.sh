#!/usr/bin/env bash
# Kernel-trace-only profile of one bench workload (fast iteration loop):
#   tools/trace.sh <workload> [extra bench args...]
# -> gpurun_out/trace_<workload>/run_kernel_stats.csv, and a compact summary
#    (kernel, calls, avg us, total us per step) on stdout.
set -euo pipefail
WL=${1:-gcounter_join}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/trace_$WL
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
STEPS=10
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 "$ROOT/bench.py" --workload "$WL" --steps $STEPS --warmup 2 --no-cpu-baseline "$@" > "$OUT/bench.json"
python3 - "$OUT/run_kernel_stats.csv" $((STEPS + 3)) <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
steps = int(sys.argv[2])
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:40]:
    print(f'{r["Name"][:90]:90s} calls {int(r["Calls"]):6d} avg {float(r["AverageNs"])/1e3:9.2f} us  per-step {float(r["TotalDurationNs"])/1e3/steps:9.2f} us')
PY
