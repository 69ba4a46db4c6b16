#!/usr/bin/env bash
# Profile one bench workload on the GPU box:
#   1. rocprofv3 --kernel-trace --stats (per-kernel durations; csv)
#   2. a --pmc FETCH_SIZE pass and 3. a --pmc WRITE_SIZE pass (separate
#      passes: FETCH_SIZE uses 3 TCC slots, WRITE_SIZE 2; never combined
#      with sys/runtime traces).
# Usage: tools/profile.sh <workload> [extra bench args...]
set -euo pipefail
WL=${1:-gcounter_join}
shift || true
ROOT=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$ROOT/gpurun_out/prof_$WL
mkdir -p "$OUT"
cd /tmp
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 "$ROOT/bench.py" --workload "$WL" --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-peaks "$@" > "$OUT/bench_trace.json"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/pmc_fetch" -o run -- \
    python3 "$ROOT/bench.py" --workload "$WL" --steps 5 --warmup 1 --no-cpu-baseline --no-e2e "$@" > "$OUT/bench_fetch.json"
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/pmc_write" -o run -- \
    python3 "$ROOT/bench.py" --workload "$WL" --steps 5 --warmup 1 --no-cpu-baseline --no-e2e "$@" > "$OUT/bench_write.json"
echo "profile $WL done"
