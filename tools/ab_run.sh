#!/bin/bash
# one GPU session of A/B experiments (edited per experiment; outputs under gpurun_out/)
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
for v in seg32 seg64; do
PAC_LIB=variants/libpacgpu_$v.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "decode or dec or reference or wav or bs" > gpurun_out/t_$v.log 2>&1 || { tail -30 gpurun_out/t_$v.log; exit 1; }
echo "$v tests: $(tail -1 gpurun_out/t_$v.log)"
done
AB_ARGS="--mode decode" bash tools/ab_bench.sh head seg32 seg64 head seg32 seg64 || exit 1
AB_ARGS="--mode decode --config 3" bash tools/ab_bench.sh head seg32 seg64 || exit 1
