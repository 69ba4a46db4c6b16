#!/bin/bash
# Server.merge() phase split (CRDT_SRV_PROF=1) and its kernel list.
mkdir -p gpurun_out/srv
CRDT_SRV_PROF=1 timeout -k 10 120 python -u tools/server_prof.py 5 > gpurun_out/srv/prof5.txt 2> gpurun_out/srv/prof5.err || { tail gpurun_out/srv/prof5.err; exit 1; }
cat gpurun_out/srv/prof5.txt; tail -5 gpurun_out/srv/prof5.err
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/srv/trace -o run -- \
    python3 $GRAFT_REPO_ROOT/bench.py --workload server_merge --steps 20 --warmup 3 --no-e2e --cpu-seconds 3 > $GRAFT_REPO_ROOT/gpurun_out/srv/bench.json || exit 1
cd $GRAFT_REPO_ROOT
cat gpurun_out/srv/bench.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['value']/1e6, d['cpu_baseline']['value']/1e6)"
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/srv/trace/run_kernel_stats.csv')))
for r in rows:
    if 'stream_' in r['Name']: continue
    print(f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4}  {r['Name'][:100]}")
PY
