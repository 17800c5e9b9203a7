# radix-8 side FFT: parity subset on the working tree (r8, 4 waves/SIMD), then A/B vs r8cap (5 waves, spills) and r4
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_numerics.py tests/test_gpu_reference.py tests/test_gpu_headline.py tests/test_gpu_master.py tests/test_gpu_sweep.py tests/test_gpu_bs.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/t14_tests.log 2>&1; echo "tests rc=$?" >> gpurun_out/t14_tests.log
tail -3 gpurun_out/t14_tests.log
grep -q "tests rc=0" gpurun_out/t14_tests.log || exit 1
AB_VARIANTS="r8cap r4" bash tools/g12.sh
AB_ENVS="PAC_SIDE_LDS_PAD=0 PAC_SIDE_LDS_PAD=8192 PAC_SIDE_LDS_PAD=22000" AB_LIB=variants/libpacgpu_r4.so bash tools/ab_env.sh > gpurun_out/t14_pad.log 2>&1
cat gpurun_out/t14_pad.log
