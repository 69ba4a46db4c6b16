mkdir -p gpurun_out/r5h
timeout -k 10 900 python -u -m pytest tests/test_gpu_merge_unsorted.py tests/test_gpu_d2_planned.py tests/test_gpu_full_configs.py -m gpu -x -q --timeout 600 --timeout-method thread > gpurun_out/r5h/tests.log 2>&1 || { tail -60 gpurun_out/r5h/tests.log; exit 1; }
tail -1 gpurun_out/r5h/tests.log
bash tools/ab_knob.sh sort.lww_gather 0 1 lww_merge_d2 3 "" 'k_lww|k_sort' || exit 1
