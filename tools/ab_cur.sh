cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for i in 1 2; do timeout -k 10 300 python3 bench.py > gpurun_out/bench_config2_s$i.json 2> gpurun_out/bench_config2_s$i.err || exit 1; grep -o '"value": [0-9.]*' gpurun_out/bench_config2_s$i.json | head -1; done
