#!/bin/bash
# OR-Set D2 run dedup staged by LDS-DMA: tests, kernel stats; minmax grid sweep.
bash tools/r03_d2.sh || exit $?
O=gpurun_out/mm; mkdir -p $O
for b in 1 2 4 8; do
  timeout -k 10 120 python bench.py --workload lww_merge_d2 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --option sort.mm_blocks_per_cu=$b > $O/b$b.json 2> $O/err || { tail -3 $O/err; exit 1; }
  echo "mm_bpc=$b $(python -c "import json; d=json.load(open('$O/b$b.json')); print(d['ms_per_step'], d['roofline']['avg_launch_us'])")"
done
bash tools/kstats.sh lww_merge_d2 --option sort.mm_blocks_per_cu=1 | grep minmax
for r in 5 64; do CRDT_SRV_PROF=1 timeout -k 10 120 python tools/server_prof.py $r > gpurun_out/srvprof_$r.txt 2>&1 || exit 1; tail -4 gpurun_out/srvprof_$r.txt; done
