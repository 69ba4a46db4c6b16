#!/bin/bash
# round 3, batch 2: D2 parity + A/B, PMC width calibration, server_merge replica sweep.
O=gpurun_out/b2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_merge_unsorted.py tests/test_gpu_sort.py -m gpu -v \
  --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $O/tests.log | head -30; exit $rc; fi
for wl in lww_merge_d2 orset_merge_d2; do
  timeout -k 10 200 python bench.py --workload $wl --steps 20 --warmup 3 --no-cpu-baseline --no-e2e > $O/$wl.json 2> $O/$wl.err || exit 1
  echo "$wl $(python -c "import json; d=json.load(open('$O/$wl.json')); print(d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])")"
done
timeout -k 10 200 python bench.py --workload orset_merge_d2 --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --option sort.or_key_only=0 > $O/or_full.json 2> $O/or_full.err || exit 1
echo "orset_merge_d2 full-tag-sort $(python -c "import json; d=json.load(open('$O/or_full.json')); print(d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'])")"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/cal_fetch -o run -- $GRAFT_REPO_ROOT/tools/mb/pmc_cal > /dev/null || exit 1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/cal_write -o run -- $GRAFT_REPO_ROOT/tools/mb/pmc_cal > /dev/null || exit 1
cd $GRAFT_REPO_ROOT
python tools/pmc_cal.py $O/cal_fetch/run_counter_collection.csv $O/cal_write/run_counter_collection.csv $O/pmc_calibration.json | head -40
for r in 5 20 50; do
  timeout -k 10 200 python bench.py --workload server_merge --steps 20 --warmup 3 --no-e2e --demo-replicas $r --cpu-seconds 3 > $O/srv_$r.json 2> $O/srv_$r.err || exit 1
  echo "server_merge $r $(python -c "import json; d=json.load(open('$O/srv_$r.json')); print(d['value'], d['ms_per_step'], d['cpu_baseline']['value'] if d['cpu_baseline'] else None, d['cpu_baseline']['cores'] if d['cpu_baseline'] else None)")"
done
