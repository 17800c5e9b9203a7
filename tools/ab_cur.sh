cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
AB_ARGS="--config 2" bash tools/ab_bench.sh base rag1 || exit 1
AB_ENV="PAC_CHUNK_BLOCKS=24576" AB_ARGS="--config 2" bash tools/ab_bench.sh base || exit 1
AB_ENV="PAC_CHUNK_BLOCKS=49152" AB_ARGS="--config 2" bash tools/ab_bench.sh base || exit 1
AB_ENV="PAC_TAIL_WIDE=1" AB_ARGS="--config 2" bash tools/ab_bench.sh base || exit 1
AB_ARGS="--config 2" bash tools/ab_bench.sh base rag1 || exit 1
AB_ENV="PAC_CHUNK_BLOCKS=24576" AB_ARGS="--config 2" bash tools/ab_bench.sh base || exit 1
AB_ENV="PAC_CHUNK_BLOCKS=49152" AB_ARGS="--config 2" bash tools/ab_bench.sh base || exit 1
