# GPU session: -m gpu tests of the working build, then an A/B of configs[2]
# between ab/libpacgpu_<A>.so and the working build (interleaved, 2 rounds)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${MEAS_TAG:-ab}
if [ -z "$NO_TESTS" ]; then
timeout -k 10 900 python -u -m pytest ${PYTEST_PATHS:-tests} -m gpu -x -q ${PYTEST_EXTRA} --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1; rc=$?; tail -2 gpurun_out/${T}_tests.log; [ $rc = 0 ] || exit $rc
fi
for r in 1 2; do
  for v in "$@" cur; do
    if [ $v = cur ]; then L=perceptual-audio-codec_amd/libpacgpu.so; else L=ab/libpacgpu_$v.so; fi
    echo -n "$v: "; PAC_LIB=$L timeout -k 10 200 python bench.py --no-cpu --steps 3 --warmup 1 ${AB_ARGS} 2>gpurun_out/${T}_$v.err | grep -o '"value": [0-9.]*\|"k_master_thr": [0-9.]*\|"k_master_lrms_spec": [0-9.]*\|"ms_per_step": [0-9.]*' | tr '\n' ' ' || exit 1
    echo
  done
done
