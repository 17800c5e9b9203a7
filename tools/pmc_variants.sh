#!/bin/bash
# PMC counters of k_master_thr for A/B library variants (ab/libpacgpu_NAME.so):
#   bash tools/pmc_variants.sh NAME...   -> gpurun_out/pmcv_NAME/
# PMCV_SET: counters (one pass), PMCV_ARGS: bench.py arguments
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
SET=${PMCV_SET:-"SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64"}
ARGS=${PMCV_ARGS:-"--no-cpu --config 2 --streams 1000 --steps 1 --warmup 0"}
for v in "$@"; do
  PAC_LIB=ab/libpacgpu_$v.so timeout -k 10 120 rocprofv3 --pmc $SET --output-format csv -d gpurun_out/pmcv_$v -o pmc -- python3 bench.py $ARGS > gpurun_out/pmcv_$v.log 2>&1 || { echo "failed: $v"; exit 1; }
done
echo PMCV_DONE
