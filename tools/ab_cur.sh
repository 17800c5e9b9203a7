cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
PAC_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29555 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu > gpurun_out/r04_rank2.json 2> gpurun_out/r04_rank2.err || { tail -20 gpurun_out/r04_rank2.err; exit 1; }
tail -1 gpurun_out/r04_rank2.json | cut -c1-400
