#!/bin/bash
# (Record of a round-4 A/B: codec.str_cache was removed after it measured
# mixed)
# Decode claims with the tables' short strings cached in LDS (codec.str_cache):
# parity under both settings, then A/B on gossip_round_wire and server_merge.
mkdir -p gpurun_out/cache
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_server_resident.py tests/test_gpu_server_errors.py \
    tests/test_gpu_gossip.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/cache/tests1.log 2>&1 || { tail -30 gpurun_out/cache/tests1.log; exit 1; }
tail -1 gpurun_out/cache/tests1.log
CRDT_TEST_OPTIONS="codec.str_cache=0" timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_server_resident.py \
    -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/cache/tests0.log 2>&1 || { tail -30 gpurun_out/cache/tests0.log; exit 1; }
tail -1 gpurun_out/cache/tests0.log
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in 0 1 0 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/cache/t$v -o run -- \
      python3 $R/bench.py --workload gossip_round_wire --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --option codec.str_cache=$v \
      > $R/gpurun_out/cache/b$v.json 2> $R/gpurun_out/cache/b$v.err || { tail -3 $R/gpurun_out/cache/b$v.err; exit 1; }
  python3 - $R/gpurun_out/cache/t$v/run_kernel_stats.csv $R/gpurun_out/cache/b$v.json $v <<'PY'
import csv, json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print("str_cache", sys.argv[3], "ms/step", d["ms_per_step"], "frac", d["roofline"]["frac"])
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_dec_claim' in r['Name']:
        print("   ", f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:60]}")
PY
done
cd $R
for v in 0 1; do
timeout -k 10 200 python3 bench.py --workload server_merge --steps 50 --warmup 5 --no-e2e --cpu-seconds 2 --option codec.str_cache=$v > gpurun_out/cache/srv$v.json || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/cache/srv$v.json').read().strip().splitlines()[-1]); print('server_merge str_cache=$v ms', d['ms_per_step'], 'M/s', round(d['value']/1e6,1), 'cpu', round(d['cpu_baseline']['value']/1e6,1))"
done
