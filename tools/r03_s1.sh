#!/bin/bash
# Round-3 GPU session 1: GPU tests, the configs[2] bench line under each tail
# placement (PAC_TAIL_MODE), the 2-rank rehearsal on one GPU, and a kernel
# trace at the bench geometry.  Outputs under gpurun_out/s1_*.
cd "${GRAFT_REPO_ROOT:-.}"
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s1_tests.log 2>&1 || { echo "gpu tests failed"; tail -5 gpurun_out/s1_tests.log; exit 1; }
echo "tests ok"
for m in ${S1_MODES:-overlap serial}; do
  PAC_TAIL_MODE=$m timeout -k 10 240 python bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/s1_bench_${m/:/}.json 2> gpurun_out/s1_bench_${m/:/}.err || { echo "bench $m failed"; exit 1; }
  echo "bench $m: $(grep -o '"value": [0-9.]*' gpurun_out/s1_bench_${m/:/}.json)"
done
[ -n "$S1_SHORT" ] && { echo S1_DONE; exit 0; }
PAC_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --streams 4000 --steps 3 --warmup 1 --no-cpu > gpurun_out/s1_rank2.json 2> gpurun_out/s1_rank2.err || { echo "2-rank rehearsal failed"; exit 1; }
echo "rank2: $(grep -o '"value": [0-9.]*' gpurun_out/s1_rank2.json)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s1_kt -o kt -- python3 bench.py --no-cpu --steps 2 --warmup 1 > gpurun_out/s1_kt.log 2>&1 || { echo "kernel trace failed"; exit 1; }
echo S1_DONE
