#!/bin/bash
# RefMerge tile pass: loads only for emitted entries (default) vs every
# in-tile entry (refmerge.load_all=1): parity, then A/B on refmerge and the
# gossip round under rocprof.
mkdir -p gpurun_out/rmld
timeout -k 10 400 python -u -m pytest tests/test_gpu_refmerge.py tests/test_gpu_refmerge_edges.py tests/test_gpu_replay_delta.py \
    tests/test_gpu_gossip.py tests/test_gpu_population.py tests/test_gpu_shard_refmerge.py -m gpu -x -q --timeout 200 --timeout-method thread \
    > gpurun_out/rmld/tests.log 2>&1 || { tail -30 gpurun_out/rmld/tests.log; exit 1; }
tail -1 gpurun_out/rmld/tests.log
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for wl in refmerge gossip_round refmerge_delta; do
for v in 0 1 0 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/rmld/t_${wl}_$v -o run -- \
      python3 $R/bench.py --workload $wl --steps 20 --warmup 3 --no-e2e --no-cpu-baseline --option refmerge.load_all=$v \
      > $R/gpurun_out/rmld/b_${wl}_$v.json 2> $R/gpurun_out/rmld/b_${wl}_$v.err || { tail -3 $R/gpurun_out/rmld/b_${wl}_$v.err; exit 1; }
  python3 - $R/gpurun_out/rmld/t_${wl}_$v/run_kernel_stats.csv $R/gpurun_out/rmld/b_${wl}_$v.json "$wl load_all=$v" <<'PY'
import csv, json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
print(sys.argv[3], "ms/step", d["ms_per_step"], "frac", d["roofline"]["frac"])
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_rm_tile' in r['Name']:
        print("   ", f"{float(r['AverageNs'])/1e3:8.1f} us x{r['Calls']:>4} {r['Name'][:50]}")
PY
done
done
