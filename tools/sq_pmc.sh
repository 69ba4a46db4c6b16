# One --pmc pass of SQ counters over a bench workload: tools/sq_pmc.sh <tag> <workload> [bench options]
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; tag=$1; wl=$2; shift 2
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_WAVES --output-format csv -d $R/gpurun_out/$tag -o run -- python3 $R/bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline "$@" > $R/gpurun_out/$tag.json
