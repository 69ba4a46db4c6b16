#!/bin/bash
# gossip_round_wire: kernel list and one step's timeline (gaps = host time).
mkdir -p gpurun_out/wire
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/wire/t -o run -- \
    python3 $R/bench.py --workload gossip_round_wire --steps 10 --warmup 2 --no-e2e --no-cpu-baseline \
    > $R/gpurun_out/wire/b.json 2> $R/gpurun_out/wire/b.err || { tail -3 $R/gpurun_out/wire/b.err; exit 1; }
python3 - $R/gpurun_out/wire/t/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'stream_' in r['Name']: continue
    print(f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:80]}")
PY
