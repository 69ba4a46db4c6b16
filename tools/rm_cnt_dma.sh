#!/bin/bash
# RefMerge count pass staged by LDS-DMA (default) against register staging (refmerge.count_dma=0)
set -o pipefail
T="tests/test_gpu_refmerge.py tests/test_gpu_refmerge_edges.py tests/test_gpu_replay_delta.py tests/test_gpu_gossip.py tests/test_gpu_server_resident.py tests/test_gpu_shard_refmerge.py tests/test_gpu_server_errors.py"
timeout -k 10 400 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > gpurun_out/rcd_t.log 2>&1 || { tail -30 gpurun_out/rcd_t.log; exit 1; }
tail -1 gpurun_out/rcd_t.log
for r in a b c; do for k in 1 0; do
  bash tools/kstats.sh rcd$k$r refmerge --option refmerge.count_dma=$k | grep k_rm_count | sed "s/^/dma$k /"
  python -c "import json; d=json.load(open('gpurun_out/ks_rcd$k$r.json')); print('dma $k', d['ms_per_step'])"
done; done
