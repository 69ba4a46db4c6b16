#!/bin/bash
# evidence: rocprofv3 --kernel-trace --stats + FETCH_SIZE / WRITE_SIZE passes per workload
# (tools/profile.sh), each step under its own time limit; stops at the first failure.
for wl in ${WLS:-shard_fold lww_merge orset_merge lww_merge_d2 orset_merge_d2 refmerge refmerge_delta gossip_round}; do
  bash tools/profile.sh $wl > gpurun_out/prof_$wl.log 2>&1 || { echo "profile $wl failed"; tail -5 gpurun_out/prof_$wl.log; exit 1; }
  echo "profiled $wl"
done
