#!/bin/bash
bash tools/kstats.sh orset_merge_d2 && bash tools/kstats.sh lww_merge_d2 && bash tools/ab_build.sh lww_merge 2 && bash tools/ab_build.sh server_merge 2 --demo-replicas 5
