#!/bin/bash
# round-3 check: selected GPU tests, then the set-merge schedule sweep.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_server_errors.py tests/test_gpu_shard_comm.py} -m gpu -v \
  --timeout 300 --timeout-method thread > gpurun_out/r03_tests.log 2>&1
rc=$?
tail -5 gpurun_out/r03_tests.log
if [ $rc -ne 0 ]; then grep -E "^E |Error|FAILED" gpurun_out/r03_tests.log | head -30; exit $rc; fi
if [ $# -gt 0 ]; then bash tools/chunk_ab.sh "$@"; exit $?; fi
exit 0
