cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t1_gputests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/t1_gputests.log; exit 1; }
tail -2 gpurun_out/t1_gputests.log
AB_ARGS="--config 2" bash tools/ab_bench.sh base new base new || exit 1
AB_ARGS="--config 1" bash tools/ab_bench.sh base new || exit 1
AB_ARGS="--config 3" bash tools/ab_bench.sh base new || exit 1
AB_ARGS="--config 4" bash tools/ab_bench.sh base new || exit 1
