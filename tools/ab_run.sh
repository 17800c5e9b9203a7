#!/bin/bash
# one GPU session of A/B experiments (edited per experiment; outputs under gpurun_out/)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
PAC_LIB=variants/libpacgpu_g8.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "decode or dec or reference or wav or bs or mono or kbd or origin" > gpurun_out/t_g8.log 2>&1 || { tail -30 gpurun_out/t_g8.log; exit 1; }
echo "g8 tests: $(tail -1 gpurun_out/t_g8.log)"
AB_ARGS="--mode decode" bash tools/ab_bench.sh head g8 head g8 || exit 1
AB_ARGS="--mode decode --config 1" bash tools/ab_bench.sh head g8 || exit 1
