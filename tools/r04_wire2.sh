#!/bin/bash
# Decode entries / pairs passes with their loads hoisted: parity, then the
# wire round's kernels.
mkdir -p gpurun_out/wire2
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py tests/test_gpu_gossip.py tests/test_gpu_server_resident.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > gpurun_out/wire2/tests.log 2>&1 || { tail -30 gpurun_out/wire2/tests.log; exit 1; }
tail -1 gpurun_out/wire2/tests.log
bash tools/r04_wire_prof.sh > gpurun_out/wire2/prof.txt 2>&1 || { tail gpurun_out/wire2/prof.txt; exit 1; }
head -12 gpurun_out/wire2/prof.txt
python3 -c "import json; d=json.loads(open('gpurun_out/wire/b.json').read().strip().splitlines()[-1]); print('wire ms', d['ms_per_step'], 'frac', d['roofline']['frac'])"
