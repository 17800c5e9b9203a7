# parity subset on the working tree, then A/B against variants/libpacgpu_base.so (configs[2], configs[1])
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_numerics.py tests/test_gpu_reference.py tests/test_gpu_headline.py tests/test_gpu_master.py tests/test_gpu_sweep.py tests/test_gpu_origin.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/t10_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/t10_tests.log
tail -3 gpurun_out/t10_tests.log
grep -q "tests rc=0" gpurun_out/t10_tests.log || exit 1
for r in 1 2; do
AB_ENVS="X=base" AB_LIB=variants/libpacgpu_base.so bash tools/ab_env.sh 2>&1 | head -1
AB_ENVS="X=new" bash tools/ab_env.sh 2>&1 | head -1
done > gpurun_out/t10_ab.log
for r in 1 2; do
AB_ARGS="--config 1" AB_ENVS="X=base1" AB_LIB=variants/libpacgpu_base.so bash tools/ab_env.sh 2>&1 | head -1
AB_ARGS="--config 1" AB_ENVS="X=new1" bash tools/ab_env.sh 2>&1 | head -1
done >> gpurun_out/t10_ab.log
cat gpurun_out/t10_ab.log
