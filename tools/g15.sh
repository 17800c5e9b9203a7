# parity subset on the working tree, then PAC_LINES_MD=0/1 on the same box (configs[2], configs[3])
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_numerics.py tests/test_gpu_reference.py tests/test_gpu_headline.py tests/test_gpu_master.py tests/test_gpu_sweep.py tests/test_gpu_continue.py tests/test_gpu_shard.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/t15_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/t15_tests.log
tail -3 gpurun_out/t15_tests.log
grep -q "tests rc=0" gpurun_out/t15_tests.log || exit 1
AB_ENVS="PAC_LINES_MD=0 PAC_LINES_MD=1" bash tools/ab_env.sh > gpurun_out/t15_ab.log 2>&1
AB_ARGS="--config 3" AB_ENVS="PAC_LINES_MD=0 PAC_LINES_MD=1" bash tools/ab_env.sh >> gpurun_out/t15_ab.log 2>&1
cat gpurun_out/t15_ab.log
