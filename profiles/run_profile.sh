#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root via gpurun).
#   kernel trace + stats, then PMC passes (instruction mix, FP64 mix, HBM bytes)
# Outputs land in gpurun_out/prof_*; the summaries worth keeping are copied
# into profiles/ by hand (profiles/rocpd_summary.py for rocpd databases).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
ARGS=${PROF_ARGS:-"--no-cpu --streams 200 --steps 2 --warmup 1"}
TAG=${PROF_TAG:-r01}
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_gfx950.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_kt -o kt -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}_kt.log 2>&1 || exit 1
for set in "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  name=$(echo $set | cut -d' ' -f1 | tr 'A-Z' 'a-z')
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/prof_${TAG}_${name} -o pmc -- python3 bench.py $ARGS > gpurun_out/prof_${TAG}_${name}.log 2>&1 || echo "pmc set failed: $set"
done
echo PROFILE_DONE
