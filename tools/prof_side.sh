set -e
mkdir -p gpurun_out
PAC_DEBUG_FLAGS=32 timeout -k 10 120 python bench.py --config 2 --steps 1 --warmup 1 > gpurun_out/ps_side.json 2> gpurun_out/ps_side.err
PAC_DEBUG_FLAGS=64 timeout -k 10 120 python bench.py --config 2 --steps 1 --warmup 1 > gpurun_out/ps_front.json 2> gpurun_out/ps_front.err
grep -A9 PAC_PROF gpurun_out/ps_side.err | tail -10
grep -A9 PAC_PROF gpurun_out/ps_front.err | tail -10
