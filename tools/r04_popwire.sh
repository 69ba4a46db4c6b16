#!/bin/bash
# crdt_population_round_wire: parity (population + codec suites), then the
# wire round native vs Python-orchestrated, and its kernels.
mkdir -p gpurun_out/popwire
timeout -k 10 400 python -u -m pytest tests/test_gpu_population.py tests/test_gpu_codec.py -m gpu -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/popwire/tests.log 2>&1 || { tail -40 gpurun_out/popwire/tests.log; exit 1; }
tail -1 gpurun_out/popwire/tests.log
for impl in native python native python; do
  CRDT_GOSSIP_IMPL=$impl timeout -k 10 200 python bench.py --workload gossip_round_wire --steps 10 --warmup 2 --no-e2e \
      --no-cpu-baseline > gpurun_out/popwire/b_$impl.json 2> gpurun_out/popwire/b_$impl.err || { tail -5 gpurun_out/popwire/b_$impl.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/popwire/b_$impl.json').read().strip().splitlines()[-1]); print('$impl', d['ms_per_step'], d['roofline']['frac'])"
done
bash tools/r04_wire_prof.sh > gpurun_out/popwire/prof.txt 2>&1 || { tail gpurun_out/popwire/prof.txt; exit 1; }
head -14 gpurun_out/popwire/prof.txt
