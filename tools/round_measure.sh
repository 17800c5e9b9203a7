#!/bin/bash
# One GPU session: the bench line of every workload + the rocprofv3 profiles
# (kernel trace + PMC passes) of master / origin / block switching, all at the
# current build.  Outputs under gpurun_out/; copy what is judged into profiles/.
#   bash tools/round_measure.sh          (run on the GPU box via gpurun)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
set -o pipefail
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.err || { echo "bench $name failed"; exit 1; }; echo "bench $name done"; }
run config2
run config1 --config 1
run config3 --config 3
run config4 --config 4
run decode --mode decode
PROF_TAG=r02_master PROF_ARGS="--no-cpu --config 2 --streams 1000 --steps 2 --warmup 1" bash profiles/run_profile.sh || exit 1
PROF_TAG=r02_origin PROF_ARGS="--no-cpu --config 1 --steps 2 --warmup 1" bash profiles/run_profile.sh || exit 1
PROF_TAG=r02_bs PROF_ARGS="--no-cpu --config 4 --streams 1000 --steps 2 --warmup 1" bash profiles/run_profile.sh || exit 1
echo MEASURE_DONE
