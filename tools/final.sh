#!/bin/bash
# Final measurement of a round, first half (GPU box via gpurun): the GPU test
# suite, every workload's bench line (CPU baseline + parity sample), the
# two-rank rehearsals (bench.py --gpus 2 spawning its ranks, and under
# torch.distributed.run as the driver launches N > 1) on the one GPU, and
# smoke(), at the current build.  The profiles are tools/prof.sh (a second
# call).  Outputs under gpurun_out/; copied into profiles/ locally.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
set -o pipefail
T=${MEAS_TAG:-r06}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gputests.log 2>&1 || { echo "gpu tests failed"; tail -20 gpurun_out/${T}_gputests.log; exit 1; }
tail -1 gpurun_out/${T}_gputests.log
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.err || { echo "bench $name failed"; tail -5 gpurun_out/bench_$name.err; exit 1; }; echo "bench $name: $(grep -o '"value": [0-9.]*' gpurun_out/bench_$name.json | head -1)"; }
run config2 --steps 20 --warmup 5
run config1 --config 1
run config3 --config 3
run config4 --config 4
run decode --mode decode
PAC_BENCH_SHARE_GPU=1 timeout -k 10 400 python3 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench_spawn2.json 2> gpurun_out/bench_spawn2.err || { echo "spawn rehearsal failed"; tail -5 gpurun_out/bench_spawn2.err; exit 1; }
echo "spawn --gpus 2 rehearsal: $(grep -o '"value": [0-9.]*\|"n_gpus": [0-9]*' gpurun_out/bench_spawn2.json | head -2 | tr '\n' ' ')"
PAC_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/bench_rank2.json 2> gpurun_out/bench_rank2.err || { echo "rank-2 rehearsal failed"; tail -5 gpurun_out/bench_rank2.err; exit 1; }
echo "torchrun rank-2 rehearsal: $(grep -o '"value": [0-9.]*\|"n_gpus": [0-9]*' gpurun_out/bench_rank2.json | head -2 | tr '\n' ' ')"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
echo FINAL_DONE
