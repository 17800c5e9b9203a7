#!/bin/bash
# A/B of environment switches on the current build in one GPU session:
#   AB_ENVS="PAC_FRONT_FAST=0 PAC_FRONT_FAST=1" bash tools/ab_env.sh    (AB_ARGS: bench arguments)
#   (several variables in one entry joined by "+": PAC_SIDE_EARLY=1+PAC_STREAM_PRIO=0121; AB_LIB: library)
cd "${GRAFT_REPO_ROOT:-.}"
for rep in 1 2; do
  for e in $AB_ENVS; do
    echo -n "$e: "; env ${AB_LIB:+PAC_LIB=$AB_LIB} ${e//+/ } timeout -k 10 120 python bench.py --no-cpu --steps 3 --warmup 1 ${AB_ARGS:---config 2} 2>&1 | grep -o '"value": [0-9.]*\|"kernels_ms": {[^}]*}' | tr '\n' ' ' || exit 1
    echo
  done
done
