#!/bin/bash
# (Record of a round-4 A/B: the sort.vec_up=2 / *_stage knobs it sets were
# removed after it measured them slower, DESIGN.md §5.5 "Round 4".)
# D2: parity of the new minmax (16-B rep chunks) and the LDS-DMA composing
# upsweep (sort.vec_up=2), then A/B timing and the dedup-apply diagnostics.
mkdir -p gpurun_out/d2ab
R=$GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_merge_unsorted.py tests/test_gpu_sort.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/d2ab/tests_vec1.log 2>&1 || { tail -20 gpurun_out/d2ab/tests_vec1.log; exit 1; }
tail -2 gpurun_out/d2ab/tests_vec1.log
CRDT_TEST_OPTIONS="sort.vec_up=2,sort.dd_stage=1,sets.lww_stage=1,sets.or_stage=1" timeout -k 10 400 python -u -m pytest tests/test_gpu_merge_unsorted.py tests/test_gpu_sort.py tests/test_gpu_vclock_sets.py \
    -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/d2ab/tests_vec2.log 2>&1 || { tail -20 gpurun_out/d2ab/tests_vec2.log; exit 1; }
tail -2 gpurun_out/d2ab/tests_vec2.log
cd /tmp && export TMPDIR=/tmp
for wl in lww_merge_d2 orset_merge_d2; do
for v in 1 2 1 2; do
  st=$(( v - 1 ))
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/d2ab/t_${wl}_$v -o run -- \
      python3 $R/bench.py --workload $wl --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --option sort.vec_up=$v --option sort.dd_stage=$st \
      > $R/gpurun_out/d2ab/b_${wl}_$v.json 2> $R/gpurun_out/d2ab/b_${wl}_$v.err || { tail -3 $R/gpurun_out/d2ab/b_${wl}_$v.err; exit 1; }
  python3 - $R/gpurun_out/d2ab/t_${wl}_$v/run_kernel_stats.csv $R/gpurun_out/d2ab/b_${wl}_$v.json "$wl vec_up=$v dd_stage=$st" <<'PY'
import csv, json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[3], "ms/step", d["ms_per_step"], "avg_launch_us", d["roofline"]["avg_launch_us"])
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_sort_minmax' in r['Name'] or 'k_sort_up_vec' in r['Name'] or 'k_dd_apply' in r['Name'] or 'k_or_rdd_apply' in r['Name']:
        print("   ", f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:60]}")
PY
done
done
for v in 0 1 0 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/d2ab/t_or_$v -o run -- \
      python3 $R/bench.py --workload orset_merge --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --option sets.or_stage=$v \
      > $R/gpurun_out/d2ab/b_or_$v.json 2> $R/gpurun_out/d2ab/b_or_$v.err || { tail -3 $R/gpurun_out/d2ab/b_or_$v.err; exit 1; }
  python3 - $R/gpurun_out/d2ab/t_or_$v/run_kernel_stats.csv $R/gpurun_out/d2ab/b_or_$v.json "orset_merge or_stage=$v" <<'PY'
import csv, json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[3], "ms/step", d["ms_per_step"], "avg_launch_us", d["roofline"]["avg_launch_us"])
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_or_write' in r['Name']:
        print("   ", f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:60]}")
PY
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/d2ab/t_lww_$v -o run -- \
      python3 $R/bench.py --workload lww_merge --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --option sets.lww_stage=$v \
      > $R/gpurun_out/d2ab/b_lww_$v.json 2> $R/gpurun_out/d2ab/b_lww_$v.err || { tail -3 $R/gpurun_out/d2ab/b_lww_$v.err; exit 1; }
  python3 - $R/gpurun_out/d2ab/t_lww_$v/run_kernel_stats.csv $R/gpurun_out/d2ab/b_lww_$v.json "lww_merge lww_stage=$v" <<'PY'
import csv, json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[3], "ms/step", d["ms_per_step"], "avg_launch_us", d["roofline"]["avg_launch_us"])
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_lww_write' in r['Name']:
        print("   ", f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:60]}")
PY
done
for d in 1 2; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/d2ab/diag$d -o run -- \
      python3 $R/bench.py --workload lww_merge_d2 --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --option sort.rdd_diag=$d \
      > $R/gpurun_out/d2ab/diag$d.json 2> $R/gpurun_out/d2ab/diag$d.err || { tail -3 $R/gpurun_out/d2ab/diag$d.err; exit 1; }
  python3 - $R/gpurun_out/d2ab/diag$d/run_kernel_stats.csv $d <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_dd_' in r['Name']:
        print("diag", sys.argv[2], f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:60]}")
PY
done
