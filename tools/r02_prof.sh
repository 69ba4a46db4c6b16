# Round-2 evidence: rocprofv3 stats + FETCH/WRITE PMC passes for the given workloads
set -e
for wl in "$@"; do bash tools/profile.sh $wl; done
