#!/bin/bash
# bench lines with the end-to-end (PCIe-inclusive) measurement, one per workload
set -o pipefail
O=gpurun_out/e2e
mkdir -p $O
for wl in ${WORKLOADS:-gcounter_join lww_merge orset_merge_d2 refmerge}; do
  timeout -k 10 200 python bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline > $O/$wl.json 2> $O/$wl.err || { tail -5 $O/$wl.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$wl.json')); print('$wl', d['ms_per_step'], d['e2e_pcie'])"
done
