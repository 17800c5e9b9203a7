# parity subset (default = front late), then A/B PAC_FRONT_LATE=0/1 on the same box
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_reference.py tests/test_gpu_headline.py tests/test_gpu_master.py tests/test_gpu_sweep.py tests/test_gpu_continue.py tests/test_gpu_bs.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/t4_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/t4_tests.log
tail -3 gpurun_out/t4_tests.log
grep -q "tests rc=0" gpurun_out/t4_tests.log || exit 1
AB_ENVS="PAC_FRONT_LATE=0 PAC_FRONT_LATE=1" bash tools/ab_env.sh > gpurun_out/t4_ab.log 2>&1
AB_ARGS="--config 3" AB_ENVS="PAC_FRONT_LATE=0 PAC_FRONT_LATE=1" bash tools/ab_env.sh >> gpurun_out/t4_ab.log 2>&1
cat gpurun_out/t4_ab.log
