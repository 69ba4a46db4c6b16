#!/bin/bash
# Host phase split of the batched Server.merge() (CRDT_SRV_PROF=1), baseline build vs in-tree build.
set -o pipefail
for b in base new; do
  if [ $b = base ]; then export CRDT_AMD_LIB=$PWD/crdt_amd/ab_base/libcrdt_amd.so; else unset CRDT_AMD_LIB; fi
  CRDT_SRV_PROF=1 timeout -k 10 120 python tools/server_prof.py > gpurun_out/srvp_$b.out 2> gpurun_out/srvp_$b.err || { tail -5 gpurun_out/srvp_$b.err; exit 1; }
  echo "== $b $(cat gpurun_out/srvp_$b.out)"
  grep srv_merge gpurun_out/srvp_$b.err | tail -3
done
