#!/bin/bash
# RefMerge tile-pass time under the fold timing diagnostics (WRONG state; timing only):
# 0 full, 1 skip the replay fold, 2 no flush, 4 no table, 5 no Atoi gather
set -e
for k in 0 1 2 4 5; do
  bash tools/kstats.sh diag$k refmerge --option refmerge.diag_fold=$k | grep -E "k_rm_tile|k_rm_count" || true
done
