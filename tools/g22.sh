#!/bin/bash
# pipelined MLD skip: the whole GPU suite, then A/B vs HEAD (configs[2], [3]) and PAC_MLD_SKIP=0
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > gpurun_out/g22_tests.log 2>&1 || { tail -30 gpurun_out/g22_tests.log; exit 1; }
tail -2 gpurun_out/g22_tests.log
AB_VARIANTS="base" bash tools/g12.sh > gpurun_out/g22.log || exit 1
AB_ENVS="PAC_MLD_SKIP=0" bash tools/ab_env.sh >> gpurun_out/g22.log || exit 1
AB_VARIANTS="base" AB_ARGS="--config 3" bash tools/g12.sh >> gpurun_out/g22.log || exit 1
cat gpurun_out/g22.log
