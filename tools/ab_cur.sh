cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
AB_ARGS="--config 2" bash tools/ab_bench.sh base tq4 tq8 base tq4 tq8 || exit 1
