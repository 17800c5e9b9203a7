#!/bin/bash
# Profiling session (GPU box via gpurun): rocprofv3 kernel traces +
# PMC passes of master / origin / block switching / decode at the bench
# geometry, at the current build.  Split from tools/round_measure.sh so that each
# gpurun call stays well inside its time limit.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
set -o pipefail
T=${MEAS_TAG:-r06}
PROF_TAG=${T}_master PROF_ARGS="--no-cpu --config 2 --steps 2 --warmup 1" bash profiles/run_profile.sh || exit 1
PROF_TAG=${T}_origin PROF_ARGS="--no-cpu --config 1 --steps 2 --warmup 1" bash profiles/run_profile.sh || exit 1
PROF_TAG=${T}_bs PROF_ARGS="--no-cpu --config 4 --steps 1 --warmup 1" bash profiles/run_profile.sh || exit 1
PROF_TAG=${T}_decode PROF_ARGS="--no-cpu --mode decode --steps 2 --warmup 1" bash profiles/run_profile.sh || exit 1
echo PROF_DONE
