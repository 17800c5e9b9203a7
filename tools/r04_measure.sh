#!/bin/bash
# Round-4 measurement session (run on the GPU box via gpurun): the GPU test
# suite, every workload's bench line (CPU baseline + parity sample), the
# rocprofv3 kernel-trace + PMC profiles of master / origin / block switching /
# decode at the bench geometry -- all at the current build.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
set -o pipefail
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_gputests.log 2>&1 || { echo "gpu tests failed"; tail -20 gpurun_out/r04_gputests.log; exit 1; }
tail -1 gpurun_out/r04_gputests.log
MEAS_TAG=r04 bash tools/round_measure.sh || exit 1
PROF_TAG=r04_decode PROF_ARGS="--no-cpu --mode decode --steps 2 --warmup 1" bash profiles/run_profile.sh || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 gpurun_out/r04_smoke.log
echo R04_DONE
