#!/bin/bash
# One-pair populations: parity, then a two-build A/B of the gossip round
# (base = the library before the one-pair kv passes, crdt_amd/ab_base), its
# kernels, and the refmerge_delta line with its one-copy state restore.
mkdir -p gpurun_out/onepair
timeout -k 10 400 python -u -m pytest tests/test_gpu_population.py tests/test_gpu_gossip.py tests/test_gpu_refmerge.py \
    tests/test_gpu_replay_delta.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/onepair/tests.log 2>&1 \
    || { tail -30 gpurun_out/onepair/tests.log; exit 1; }
tail -1 gpurun_out/onepair/tests.log
bash tools/ab_build.sh gossip_round 3 || exit 1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/onepair/t -o run -- \
    python3 $R/bench.py --workload gossip_round --steps 20 --warmup 3 --no-e2e --no-cpu-baseline > $R/gpurun_out/onepair/b.json 2>&1 || exit 1
python3 - $R/gpurun_out/onepair/t/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_rm' in r['Name'] or 'k_pop' in r['Name']:
        print(f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:60]}")
PY
cd $R
timeout -k 10 200 python3 bench.py --workload refmerge_delta --steps 20 --warmup 3 --no-e2e --no-cpu-baseline > gpurun_out/onepair/delta.json || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/onepair/delta.json').read().strip().splitlines()[-1]); print('refmerge_delta', d['ms_per_step'], d['roofline']['frac'])"
