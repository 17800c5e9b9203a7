# bench lines of every workload (no CPU baseline) at the current build
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for a in "--config 2" "--config 1" "--config 3" "--config 4" "--mode decode"; do
  echo -n "$a: "; timeout -k 10 200 python bench.py --no-cpu --steps 3 --warmup 1 $a 2>&1 | grep -o '"value": [0-9.]*\|"kernels_ms": {[^}]*}' | tr '\n' ' ' || exit 1; echo
done > gpurun_out/t11.log
cat gpurun_out/t11.log
