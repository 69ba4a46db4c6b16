set -o pipefail
mkdir -p gpurun_out/orab
timeout -k 10 300 python -u -m pytest tests/test_gpu_vclock_sets.py -x -q --timeout 120 --timeout-method thread > gpurun_out/orab/t.log 2>&1 || { tail -30 gpurun_out/orab/t.log; exit 1; }
tail -2 gpurun_out/orab/t.log
for k in 1 17 1 17; do
timeout -k 10 200 python bench.py --workload orset_merge --no-cpu-baseline --option sets.knobs=$k > gpurun_out/orab/b$k.json 2>gpurun_out/orab/b.err || { tail -5 gpurun_out/orab/b.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/orab/b$k.json')); print('knobs $k', d['ms_per_step'], d['roofline']['frac'])"
done
