#!/bin/bash
# One GPU session: the bench line of every workload (with the CPU baseline
# and the bench's own parity sample) + the rocprofv3 profiles (kernel trace +
# PMC passes) of master / origin / block switching at the bench geometry, all
# at the current build.  Outputs under gpurun_out/; copy what is judged into
# profiles/.   bash tools/round_measure.sh   (run on the GPU box via gpurun)
#   MEAS_TAG: profile tag prefix (default r05)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
set -o pipefail
T=${MEAS_TAG:-r05}
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.err || { echo "bench $name failed"; exit 1; }; echo "bench $name: $(grep -o '"value": [0-9.]*' gpurun_out/bench_$name.json)"; }
run config2 --steps 5 --warmup 1
run config1 --config 1
run config3 --config 3
run config4 --config 4
run decode --mode decode
PROF_TAG=${T}_master PROF_ARGS="--no-cpu --config 2 --steps 2 --warmup 1" bash profiles/run_profile.sh || exit 1
PROF_TAG=${T}_origin PROF_ARGS="--no-cpu --config 1 --steps 2 --warmup 1" bash profiles/run_profile.sh || exit 1
PROF_TAG=${T}_bs PROF_ARGS="--no-cpu --config 4 --steps 1 --warmup 1" bash profiles/run_profile.sh || exit 1
echo MEASURE_DONE
