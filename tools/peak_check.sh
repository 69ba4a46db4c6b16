#!/bin/bash
# GPU check of the self-measured peak kernels: their test, then the default bench line and one set line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_counters.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 200 python bench.py --steps 20 --warmup 3 > gpurun_out/b_sf.json 2> gpurun_out/b_sf.err || { tail -5 gpurun_out/b_sf.err; exit 1; }
timeout -k 10 200 python bench.py --workload lww_merge --no-cpu-baseline > gpurun_out/b_lww.json 2> gpurun_out/b_lww.err || { tail -5 gpurun_out/b_lww.err; exit 1; }
cat gpurun_out/b_sf.json gpurun_out/b_lww.json | python -c '
import sys, json
for l in sys.stdin:
    d = json.loads(l); r = d["roofline"]
    print(d["config"]["workload"][:40], r["frac"], r["frac_of_copy_peak"], r["measured_peak"])'
