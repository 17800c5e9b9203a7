cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_numerics.py tests/test_gpu_reference.py tests/test_gpu_headline.py tests/test_gpu_master.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/t2_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/t2_tests.log
tail -5 gpurun_out/t2_tests.log
grep -q "tests rc=0" gpurun_out/t2_tests.log || exit 1
AB_ENVS="PAC_SIDE_WAVE=0 PAC_SIDE_WAVE=1" bash tools/ab_env.sh > gpurun_out/t2_ab.log 2>&1 || exit 1
AB_ENVS="PAC_SIDE_WAVE=1" AB_LIB=variants/libpacgpu_side2.so bash tools/ab_env.sh >> gpurun_out/t2_ab.log 2>&1
cat gpurun_out/t2_ab.log
