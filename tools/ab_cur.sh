cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
AB_ARGS="--config 2" bash tools/ab_bench.sh base nt1 nt2 fr fr4 cut57 base nt1 nt2 fr fr4 cut57 || exit 1
AB_ENV="PAC_TAIL_MODE=serial" AB_ARGS="--config 2" bash tools/ab_bench.sh base || exit 1
PAC_LIB=variants/libpacgpu_cut57.so timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t_cut57.log 2>&1; tail -2 gpurun_out/t_cut57.log
