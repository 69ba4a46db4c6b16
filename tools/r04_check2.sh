#!/bin/bash
# Round 4: population undo test, gossip_round bench through the C-ABI vs the
# Python orchestration (A/B in one call), then the native round's profile.
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_population.py -m gpu -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/r4_pop.log 2>&1 || { tail -30 gpurun_out/r4_pop.log; exit 1; }
tail -3 gpurun_out/r4_pop.log
for impl in native python native python; do
  CRDT_GOSSIP_IMPL=$impl timeout -k 10 300 python -u bench.py --workload gossip_round --steps 30 --warmup 3 \
      --no-cpu-baseline --no-e2e > gpurun_out/r4_gossip_$impl.json 2> gpurun_out/r4_gossip_$impl.err || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/r4_gossip_$impl.json').read())
print('$impl', d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
done
bash tools/profile.sh gossip_round || exit $?
python3 tools/pmc_summary.py gossip_round k_rm_count,k_rm_tile,k_rm_split,k_rm_scan,k_rm_plan,k_slot_final,k_scan_tsums,k_out_off,k_rm_ntiles,k_pop_bounds r04 > gpurun_out/r4_gossip_pmc.txt 2>&1 || { cat gpurun_out/r4_gossip_pmc.txt; exit 1; }
grep -E "traffic_over|hbm_bytes|avg" gpurun_out/r4_gossip_pmc.txt
cp profiles/r04_gossip_round_* profiles/traffic.json gpurun_out/
cut -d, -f1-5 profiles/r04_gossip_round_kernel_stats.csv | grep -v stream_ | head -14
