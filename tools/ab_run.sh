#!/bin/bash
# one GPU session of A/B experiments (edited per experiment; outputs under gpurun_out/)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "decode or dec or reference or wav" > gpurun_out/t_dec.log 2>&1 || { tail -30 gpurun_out/t_dec.log; exit 1; }
tail -2 gpurun_out/t_dec.log
AB_ARGS="--mode decode" bash tools/ab_bench.sh tile stab tile stab || exit 1
