#!/bin/bash
bash tools/kstats.sh lww_merge_d2 > gpurun_out/d2_lww.txt && bash tools/kstats.sh orset_merge_d2 > gpurun_out/d2_or.txt && bash tools/kstats.sh server_merge --demo-replicas 5 > gpurun_out/srv.txt
rc=$?; cat gpurun_out/d2_lww.txt gpurun_out/d2_or.txt gpurun_out/srv.txt; exit $rc
