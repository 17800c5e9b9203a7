#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root via gpurun):
#   1. rocprofv3 --kernel-trace --stats of the bench command
#   2. separate --pmc passes (no tracing domains mixed in): instruction mix,
#      FP64 mix, stall/LDS counters, FETCH_SIZE, WRITE_SIZE
# Outputs land in gpurun_out/prof_<TAG>_*; then, locally:
#   python profiles/summarize_pmc.py gpurun_out/prof_<TAG> <blocks_total> > profiles/<TAG>_pmc.json
#   cp gpurun_out/prof_<TAG>_kt/kt_kernel_stats.csv profiles/<TAG>_kernel_stats.csv
# TAG names the round and the profile, e.g. r02_master / r02_origin (bench.py
# looks for profiles/r*_<profile>_pmc.json).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
# default: the bench's own geometry (configs[2], 10^4 streams x 1000 blocks,
# chunks of S = 6 blocks per stream), so the trace's per-kernel totals are
# comparable with the bench line's kernels_ms
ARGS=${PROF_ARGS:-"--no-cpu --config 2 --steps 2 --warmup 1"}
TAG=${PROF_TAG:-r03_master}
LIM=${PROF_LIMIT:-240}
timeout -k 10 $LIM rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_kt -o kt -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}_kt.log 2>&1 || { echo "kernel trace failed"; exit 1; }
for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  name=$(echo $set | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  timeout -k 10 $LIM rocprofv3 --pmc $set --output-format csv -d gpurun_out/prof_${TAG}_${name} -o pmc -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}_${name}.log 2>&1 || { echo "pmc set failed: $set"; exit 1; }
done
echo PROFILE_DONE
