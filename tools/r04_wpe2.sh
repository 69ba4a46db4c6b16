#!/bin/bash
# device decode claim pass held to 8 waves per SIMD (amdgpu_waves_per_eu(8):
# SGPR spills into VGPR lanes instead of 7 waves): codec / population / server parity, then
# alternating bench lines against crdt_amd/ab_base.
set -o pipefail
OUT=gpurun_out/wpe2; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_population.py tests/test_gpu_server_resident.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 bash tools/ab_build.sh gossip_round_wire 3
