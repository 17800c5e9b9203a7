#!/bin/bash
# kernels_ms of one bench line for A/B builds: bash tools/kms.sh "<bench args>" NAME...  (cur = the working build)
cd "${GRAFT_REPO_ROOT:-.}"
ARGS=$1; shift
for v in "$@"; do
  if [ $v = cur ]; then L=perceptual-audio-codec_amd/libpacgpu.so; else L=ab/libpacgpu_$v.so; fi
  echo "$v: $(PAC_LIB=$L timeout -k 10 200 python bench.py --no-cpu $ARGS 2>/dev/null | python3 -c 'import json,sys; d=json.loads(sys.stdin.read().strip().split("\n")[-1]); print(round(d["value"]/1e6,3), {k: round(v,1) for k,v in d["kernels_ms"].items()})')" || exit 1
done
