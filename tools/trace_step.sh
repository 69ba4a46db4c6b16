#!/bin/bash
# Kernel + memory-copy timeline of a bench workload's last step (no counters):
# tools/trace_step.sh <workload> [bench args...] -> gpurun_out/trace_<wl>/ and a summary (tools/timeline.py)
wl=$1; shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/trace_$wl; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CRDT_TRACE_MARK=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O -o run -- \
  python3 $R/bench.py --workload $wl --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-peaks "$@" > $O/bench.json 2> $O/bench.err \
  || { tail -5 $O/bench.err; exit 1; }
python3 $R/tools/timeline.py $O 5 --seq
