#!/bin/bash
# Round 4: the look-back microbenchmark (XCD-chunked vs blockIdx order vs
# reduce/scan/apply), then rocprofv3 stats + FETCH/WRITE PMC of the default
# gossip round (in-place pulls, fused kv output).
mkdir -p gpurun_out
ROOT=$(pwd)
timeout -k 10 120 ./tools/mb/lookback 4096 > gpurun_out/r4_lookback.txt 2>&1 || { cat gpurun_out/r4_lookback.txt; exit 1; }
cat gpurun_out/r4_lookback.txt
timeout -k 10 120 ./tools/mb/lookback 16384 > gpurun_out/r4_lookback_64m.txt 2>&1 || { cat gpurun_out/r4_lookback_64m.txt; exit 1; }
cat gpurun_out/r4_lookback_64m.txt
bash tools/profile.sh gossip_round || exit $?
python3 tools/pmc_summary.py gossip_round k_rm_count,k_rm_tile,k_rm_split,k_rm_scan,k_rm_plan,k_slot_final,k_scan_tsums,k_out_off,k_rm_ntiles r04 > gpurun_out/r4_gossip_pmc.txt 2>&1 || { cat gpurun_out/r4_gossip_pmc.txt; exit 1; }
tail -30 gpurun_out/r4_gossip_pmc.txt
cp profiles/r04_gossip_round_* profiles/traffic.json gpurun_out/ 2>/dev/null
head -30 profiles/r04_gossip_round_kernel_stats.csv
