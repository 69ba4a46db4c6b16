#!/bin/bash
bash tools/kstats.sh gossip_round_wire > /dev/null; python3 - <<'PY'
import csv
rows = list(csv.DictReader(open('gpurun_out/ks_gossip_round_wire/run_kernel_trace.csv')))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'k_rm_plan_small' in r['Kernel_Name']]
s, e = idx[-2] + 1, idx[-1] + 1
prev = None
for r in rows[s:e]:
    st, en = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    print(f"{(st - prev) / 1e3 if prev else 0:8.1f} {(en - st) / 1e3:8.1f}  {r['Kernel_Name'][:60]}")
    prev = en
PY
