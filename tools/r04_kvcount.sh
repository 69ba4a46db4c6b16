#!/bin/bash
# (Record of a round-4 A/B; the change it measured was reverted)
# KV count pass with the kv range loads issued before the merge: parity, then
# a two-build A/B on the gossip round (base = HEAD's library in crdt_amd/ab_base).
mkdir -p gpurun_out/kvcount
timeout -k 10 400 python -u -m pytest tests/test_gpu_gossip.py tests/test_gpu_population.py tests/test_gpu_refmerge.py \
    tests/test_gpu_server_resident.py tests/test_gpu_refmerge_edges.py -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/kvcount/tests.log 2>&1 || { tail -30 gpurun_out/kvcount/tests.log; exit 1; }
tail -1 gpurun_out/kvcount/tests.log
bash tools/ab_build.sh gossip_round 3 || exit 1
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/kvcount/t -o run -- \
    python3 $R/bench.py --workload gossip_round --steps 20 --warmup 3 --no-e2e --no-cpu-baseline > $R/gpurun_out/kvcount/b.json 2>&1 || exit 1
python3 - $R/gpurun_out/kvcount/t/run_kernel_stats.csv <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_rm' in r['Name']:
        print(f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:60]}")
PY
