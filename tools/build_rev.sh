#!/bin/bash
# Build ab/libpacgpu_NAME.so from the sources of git revision REV
# (A/B against the working tree):  bash tools/build_rev.sh NAME REV
set -e
cd "$(dirname "$0")/.."
d=$(mktemp -d)
git archive "$2" perceptual-audio-codec_amd/csrc include | tar -x -C "$d"
mkdir -p ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Wno-unused-value -Wno-pass-failed \
  -Wno-unused-result -o ab/libpacgpu_$1.so "$d/perceptual-audio-codec_amd/csrc/pac_abi.hip"
rm -rf "$d"
echo ab/libpacgpu_$1.so
