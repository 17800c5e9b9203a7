#!/bin/bash
# one GPU session (edited per experiment; outputs under gpurun_out/)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.err || { echo "bench $name failed"; tail -5 gpurun_out/bench_$name.err; exit 1; }; echo "bench $name: $(grep -o '"value": [0-9.]*' gpurun_out/bench_$name.json | head -1)"; }
run config2 --steps 5 --warmup 1
run config1 --config 1
run config3 --config 3
run config4 --config 4
run decode --mode decode
echo BENCH_DONE
