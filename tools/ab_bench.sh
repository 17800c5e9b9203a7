#!/bin/bash
# A/B of library variants in one GPU session: bash tools/ab_bench.sh NAME... (ab/libpacgpu_NAME.so)
# AB_ARGS: bench.py arguments (default --config 1); AB_ENV: extra environment (e.g. PAC_LRMS_ASYNC=0)
cd $GRAFT_REPO_ROOT
for v in "$@"; do
  echo -n "$v: "; env $AB_ENV PAC_LIB=ab/libpacgpu_$v.so timeout -k 10 120 python bench.py --no-cpu --steps 3 --warmup 1 ${AB_ARGS:---config 1} 2>&1 | grep -o '"value": [0-9.]*\|"kernels_ms": {[^}]*}' | tr '\n' ' ' || exit 1
  echo
done
