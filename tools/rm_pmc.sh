# SQ counters (LDS bank conflicts, wait breakdown) of the RefMerge passes, one --pmc pass
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/rmpmc -o run -- python3 $R/bench.py --workload ${1:-refmerge} --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/rmpmc.json
