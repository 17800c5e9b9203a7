#!/bin/bash
# GPU tests, then bench lines: configs[2] (default) and any CHECK_CONFIGS
# (e.g. "3 4 1"); outputs gpurun_out/chk_*.json
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
if [ -z "$CHECK_NOTEST" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/chk_tests.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/chk_tests.log; exit 1; }
  echo "tests: $(tail -1 gpurun_out/chk_tests.log)"
fi
for c in 2 $CHECK_CONFIGS; do
  timeout -k 10 300 python bench.py --no-cpu --config $c $CHECK_ARGS > gpurun_out/chk_c$c.json 2> gpurun_out/chk_c$c.err || { echo "bench config $c failed"; tail -5 gpurun_out/chk_c$c.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/chk_c$c.json'));print('config $c', round(d['value']/1e6,3),'M/s', round(d['ms_per_step'],1),'ms', {k:round(v,1) for k,v in d['kernels_ms'].items()})"
done
echo CHECK_DONE
