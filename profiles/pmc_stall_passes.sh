cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
A="--no-cpu --streams 100 --steps 1 --warmup 0"
for f in 0 1; do
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_VALU" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"; do
  n=$(echo $set | cut -d' ' -f1 | tr A-Z a-z)
  PAC_DEBUG_FLAGS=$f timeout -k 10 200 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc2_${f}_$n -o p -- python3 bench.py $A > gpurun_out/pmc2_${f}_$n.log 2>&1 || echo fail $set
done; done
