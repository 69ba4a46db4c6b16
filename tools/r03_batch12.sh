#!/bin/bash
bash tools/r03_batch10.sh || exit $?
bash tools/r03_batch11.sh || exit $?
for d in 1 2 3; do bash tools/kstats.sh orset_merge_d2 --option sort.rdd_diag=$d | grep rdd | sed "s/^/diag=$d /"; done
