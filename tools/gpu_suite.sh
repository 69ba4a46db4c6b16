#!/bin/bash
# One GPU call: the -m gpu suite, then (only if pytest ended normally: all
# passed, or ordinary test failures) the default bench line.  Any other exit
# status (timeout, abort, segfault) stops the script: nothing more runs on the GPU.
# usage: tools/gpu_suite.sh [pytest selection...]
mkdir -p gpurun_out
sel=${@:-tests}
timeout -k 10 1000 python -u -m pytest $sel -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/tests.log 2>&1
rc=$?
tail -5 gpurun_out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest exit $rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
exit $(( rc > brc ? rc : brc ))
