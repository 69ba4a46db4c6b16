#!/bin/bash
# D2 kernels after LDS-DMA staging of the run-aligned dedup; server merge overhead A/B; affected GPU tests
bash tools/kstats.sh orset_merge_d2 > gpurun_out/b6_or.txt && bash tools/kstats.sh lww_merge_d2 > gpurun_out/b6_lww.txt && \
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_merge_unsorted.py tests/test_gpu_sort.py tests/test_gpu_codec.py tests/test_gpu_server_resident.py tests/test_gpu_server_errors.py > gpurun_out/b6_tests.txt 2>&1 && \
bash tools/ab_build.sh server_merge 2 --demo-replicas 5 > gpurun_out/b6_ab.txt 2>&1; rc=$?; tail -3 gpurun_out/b6_tests.txt; cat gpurun_out/b6_or.txt gpurun_out/b6_lww.txt gpurun_out/b6_ab.txt; exit $rc
