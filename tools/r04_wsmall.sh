#!/bin/bash
# Wire round (1000 bodies): the one-pass small-body decode forced (codec.small=2)
# against the multi-pass form it takes by default at this body count.
mkdir -p gpurun_out/wsmall
for v in 1 2 1 2; do
  timeout -k 10 200 python bench.py --workload gossip_round_wire --steps 10 --warmup 2 --no-e2e --no-cpu-baseline \
      --option codec.small=$v > gpurun_out/wsmall/b$v.json 2> gpurun_out/wsmall/b$v.err || { tail -5 gpurun_out/wsmall/b$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/wsmall/b$v.json').read().strip().splitlines()[-1]); print('codec.small=$v', d['ms_per_step'], d['roofline']['frac'])"
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/wsmall/t -o run -- \
    python3 $R/bench.py --workload gossip_round_wire --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --option codec.small=2 \
    > $R/gpurun_out/wsmall/bt.json 2>&1 || exit 1
python3 - $R/gpurun_out/wsmall/t/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_dec' in r['Name'] or 'k_scan' in r['Name']:
        print(f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:60]}")
PY
