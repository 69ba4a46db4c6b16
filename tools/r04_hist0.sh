#!/bin/bash
# (Record of a round-4 A/B: sort.lww_hist0 and its kernels were removed after it
# measured neutral)
# Fused LWW D2 without the composing upsweep (sort.lww_hist0): parity, then
# A/B under rocprof.
mkdir -p gpurun_out/hist0
timeout -k 10 400 python -u -m pytest tests/test_gpu_merge_unsorted.py tests/test_gpu_sort.py tests/test_gpu_full_configs.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/hist0/tests.log 2>&1 || { tail -30 gpurun_out/hist0/tests.log; exit 1; }
tail -1 gpurun_out/hist0/tests.log
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in 0 1 0 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/hist0/t$v -o run -- \
      python3 $R/bench.py --workload lww_merge_d2 --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --option sort.lww_hist0=$v \
      > $R/gpurun_out/hist0/b$v.json 2> $R/gpurun_out/hist0/b$v.err || { tail -3 $R/gpurun_out/hist0/b$v.err; exit 1; }
  python3 - $R/gpurun_out/hist0/t$v/run_kernel_stats.csv $R/gpurun_out/hist0/b$v.json $v <<'PY'
import csv, json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print("lww_hist0", sys.argv[3], "ms/step", d["ms_per_step"], "frac", d["roofline"]["frac"])
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_sort' in r['Name'] or 'k_dd' in r['Name']:
        print("   ", f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:60]}")
PY
done
