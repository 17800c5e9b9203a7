#!/bin/bash
# Phase clocks of k_master_thr (PAC_DEBUG_FLAGS=128) at the bench geometry:
# needs the phase-clock build first (compiled out of the product):
#   python tools/build_variant.py thrprof perceptual-audio-codec_amd/csrc/pac_master.hip '#include "pac_bs.h"' $'#include "pac_bs.h"\n#define PAC_THR_PROF'
# marks 0 start, 1 variant spectrum, 2 maskers + lists + scans, 3 rows (wave
# end), 4 after the barrier, 5-7 the second variant, 8 end
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
PAC_LIB=ab/libpacgpu_thrprof.so PAC_DEBUG_FLAGS=128 timeout -k 10 120 python bench.py --no-cpu --config 2 --steps 1 --warmup 1 > gpurun_out/pt_thr.json 2> gpurun_out/pt_thr.err || exit 1
grep -A9 PAC_PROF gpurun_out/pt_thr.err | tail -10
