#!/bin/bash
# Device decode claims: both home entries looked up at once (new) against
# the two claims in turn (crdt_amd/ab_base): codec / population / gossip /
# server parity, then alternating wire-round and server_merge bench lines.
set -o pipefail
OUT=gpurun_out/claim; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_population.py tests/test_gpu_server_resident.py tests/test_gpu_gossip.py -m gpu -x -q \
    --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 bash tools/ab_build.sh gossip_round_wire 3 || exit 1
timeout -k 10 600 bash tools/ab_build.sh server_merge 2 || exit 1
