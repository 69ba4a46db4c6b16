#!/bin/bash
# Kernel timeline of the server_merge bench step (one step's kernels, durations and gaps).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/srv -o run -- \
  python3 $R/bench.py --workload server_merge --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/srv.json
python3 - $R/gpurun_out/srv/run_kernel_trace.csv <<'PY'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r['Start_Timestamp']))
# the last 1/10 of the kernels ~ one step
n = len(rows)
step = rows[-n // 12:]
t0 = int(step[0]['Start_Timestamp']); prev = t0
for r in step:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(f"{(s - t0) / 1e3:8.1f} gap {(s - prev) / 1e3:6.1f} dur {(e - s) / 1e3:6.1f}  {r['Kernel_Name'][:60]}")
    prev = e
PY
