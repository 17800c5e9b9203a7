cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_mldm.log 2>&1; tail -2 gpurun_out/t_mldm.log
AB_ARGS="--config 2" bash tools/ab_bench.sh base mldm base mldm || exit 1
AB_ARGS="--config 3" bash tools/ab_bench.sh base mldm || exit 1
AB_ARGS="--config 4" bash tools/ab_bench.sh base mldm || exit 1
