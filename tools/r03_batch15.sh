#!/bin/bash
for d in 1 2; do bash tools/kstats.sh lww_merge_d2 --option sort.rdd_diag=$d | grep dd_apply | sed "s/^/diag=$d /"; done
