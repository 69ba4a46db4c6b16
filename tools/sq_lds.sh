#!/bin/bash
# One --pmc pass of SQ wait / LDS counters over a bench workload: tools/sq_lds.sh <tag> <workload> [bench args]
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; tag=$1; wl=$2; shift 2
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/sq_$tag -o run -- python3 $R/bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline "$@" > $R/gpurun_out/sq_$tag.json
python3 - $R/gpurun_out/sq_$tag/run_counter_collection.csv <<'PY'
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r['Kernel_Name'][:40]
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, d in acc.items():
    if 'crdt' not in k: continue
    wc = d.get('SQ_WAVE_CYCLES', 1) or 1
    print(k, {c: round(v / wc, 3) if c != 'SQ_WAVE_CYCLES' else v for c, v in sorted(d.items())})
PY
