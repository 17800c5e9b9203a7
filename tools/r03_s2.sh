#!/bin/bash
# Round-3 GPU session 2: the other workloads' bench lines at the current
# build, and masking-row statistics (-DPAC_ROWPROF variant) of configs[2]
# vs configs[3] (the real-audio per-block threshold cost).
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > gpurun_out/s2_$name.json 2> gpurun_out/s2_$name.err || { echo "bench $name failed"; exit 1; }; echo "$name: $(grep -o '"value": [0-9.]*' gpurun_out/s2_$name.json)"; }
run config3 --config 3 --no-cpu
run config1 --config 1 --no-cpu
run config4 --config 4 --no-cpu
run decode --mode decode --no-cpu
PAC_LIB=variants/libpacgpu_rowprof.so timeout -k 10 200 python3 bench.py --no-cpu --config 2 --streams 1000 --steps 1 --warmup 0 > gpurun_out/s2_rowprof2.json 2> gpurun_out/s2_rowprof2.err || exit 1
PAC_LIB=variants/libpacgpu_rowprof.so timeout -k 10 200 python3 bench.py --no-cpu --config 3 --copies 100 --steps 1 --warmup 0 > gpurun_out/s2_rowprof3.json 2> gpurun_out/s2_rowprof3.err || exit 1
grep ROWPROF gpurun_out/s2_rowprof2.err | tail -2
grep ROWPROF gpurun_out/s2_rowprof3.err | tail -3
echo S2_DONE
