#!/bin/bash
# one GPU session (edited per experiment; outputs under gpurun_out/)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/chk_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/chk_tests.log; exit 1; }
echo "tests: $(tail -1 gpurun_out/chk_tests.log)"
timeout -k 10 200 python -c 'import __graft_entry__ as g; g.smoke()' > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
echo "smoke ok"
T=r03
PROF_TAG=${T}_master PROF_ARGS="--no-cpu --config 2 --steps 2 --warmup 1" bash profiles/run_profile.sh || exit 1
PROF_TAG=${T}_origin PROF_ARGS="--no-cpu --config 1 --steps 2 --warmup 1" bash profiles/run_profile.sh || exit 1
PROF_TAG=${T}_bs PROF_ARGS="--no-cpu --config 4 --steps 1 --warmup 1" bash profiles/run_profile.sh || exit 1
PROF_TAG=${T}_decode PROF_ARGS="--no-cpu --mode decode --steps 2 --warmup 1" bash profiles/run_profile.sh || exit 1
echo PROFILES_DONE
