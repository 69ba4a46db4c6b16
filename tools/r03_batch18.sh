#!/bin/bash
# decode micro-check first (fast, stops early on a failure), then the round evidence
timeout -k 10 300 python -u -m pytest tests/test_gpu_codec.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/codec_tests.log 2>&1
rc=$?; tail -2 gpurun_out/codec_tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" gpurun_out/codec_tests.log | head -30; exit $rc; fi
bash tools/round_evidence.sh
