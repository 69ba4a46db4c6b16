#!/bin/bash
# Server.merge() end to end against the C restatement on the host's CPU share, by replica count.
O=${SRV_CROSS_OUT:-gpurun_out/srv_cross}; mkdir -p $O
for r in 5 20 64 160; do
  timeout -k 10 240 python bench.py --workload server_merge --demo-replicas $r --steps 20 --warmup 3 --cpu-seconds 4 --no-e2e > $O/r$r.json 2> $O/r$r.err || { tail -3 $O/r$r.err; exit 1; }
  python - $O/r$r.json $r <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); c = d["cpu_baseline"]
print(f"replicas={sys.argv[2]} gpu {d['value']/1e6:.1f} M/s ({d['ms_per_step']:.3f} ms/step)  cpu {c['value']/1e6:.1f} M/s on {c['cores']} threads  ratio {d['value']/c['value']:.2f}")
PY
done
