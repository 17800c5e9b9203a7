#!/bin/bash
# one GPU session of A/B experiments (edited per experiment; outputs under gpurun_out/)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
PAC_LIB=variants/libpacgpu_fsplit2.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "bs or kbd or mono or master or reference" > gpurun_out/t_fsplit.log 2>&1 || { tail -30 gpurun_out/t_fsplit.log; exit 1; }
echo "fsplit tests: $(tail -1 gpurun_out/t_fsplit.log)"
AB_ARGS="--config 4" bash tools/ab_bench.sh head fsplit2 fsplit head fsplit2 fsplit || exit 1
AB_ARGS="--config 2" bash tools/ab_bench.sh head fsplit2 || exit 1
