#!/bin/bash
# one GPU session of A/B experiments (edited per experiment; outputs under gpurun_out/)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
PAC_LIB=variants/libpacgpu_wide.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "decode or dec or reference or wav or bs or origin" > gpurun_out/t_wide.log 2>&1 || { tail -30 gpurun_out/t_wide.log; exit 1; }
echo "wide tests: $(tail -1 gpurun_out/t_wide.log)"
AB_ARGS="--mode decode" bash tools/ab_bench.sh head wide head wide || exit 1
AB_ARGS="--mode decode --config 3" bash tools/ab_bench.sh head wide || exit 1
