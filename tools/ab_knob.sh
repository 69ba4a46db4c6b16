#!/bin/bash
# A/B of one kernel knob (crdt_set_option) on the GPU box, in one call:
#   1. optional parity: the selected -m gpu tests with the knob set to B
#      (CRDT_TEST_OPTIONS), so a variant is never timed before it is bit-exact;
#   2. per workload, PAIRS alternating pairs of bench lines A / B under
#      rocprofv3 --kernel-trace --stats, printing ms per step, the step's
#      HIP-event average and the kernels whose names match KERNELS.
# Every GPU step runs under its own time limit; the script stops at the first
# failure (nothing more runs on the GPU after a timeout or a crash).
#
# usage: tools/ab_knob.sh KNOB A B "WORKLOADS" [PAIRS] [TESTS] [KERNELS]
#   KNOB      option name, e.g. sets.lww_parts (the knob's A value is the default)
#   A, B      the two values
#   WORKLOADS bench workloads, e.g. "lww_merge orset_merge"
#   PAIRS     A/B pairs per workload (default 2)
#   TESTS     pytest selection run with KNOB=B first ("" = skip)
#   KERNELS   regex of kernel names to print (default: all with >= 2 % of the step)
# e.g. tools/ab_knob.sh sort.or_lookback 1 0 orset_merge_d2 3 tests/test_gpu_merge_unsorted.py 'k_or_'
set -o pipefail
knob=$1; va=$2; vb=$3; wls=$4; pairs=${5:-2}; tests=${6:-}; kre=${7:-}
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/ab_${knob//./_}; mkdir -p $O
if [ -n "$tests" ]; then
  (cd $R && CRDT_AMD_DIAG=1 CRDT_TEST_OPTIONS="$knob=$vb" timeout -k 10 600 python -u -m pytest $tests -m gpu -x -q \
      --timeout 300 --timeout-method thread > $O/tests_$vb.log 2>&1) || { tail -30 $O/tests_$vb.log; exit 1; }
  tail -1 $O/tests_$vb.log
fi
cd /tmp && export TMPDIR=/tmp
for wl in $wls; do
  for p in $(seq $pairs); do
    for v in $va $vb; do
      t=$O/${wl}_${v}_$p
      timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $t -o run -- \
          python3 $R/bench.py --workload $wl --steps 10 --warmup 2 --no-e2e --no-cpu-baseline --no-peaks --option $knob=$v \
          > $t.json 2> $t.err || { tail -3 $t.err; exit 1; }
      python3 - $t/run_kernel_stats.csv $t.json "$wl $knob=$v #$p" "$kre" <<'PY'
import csv, json, re, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[3], "ms/step", d["ms_per_step"], "avg_launch_us", d["roofline"]["avg_launch_us"], "frac", d["roofline"]["frac"])
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows) or 1.0
for r in rows:
    if (sys.argv[4] and re.search(sys.argv[4], r["Name"])) or (not sys.argv[4] and float(r["TotalDurationNs"]) / tot >= 0.02):
        print("   ", f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:70]}")
PY
    done
  done
done
