# A/B: variants vs the current build (configs[2]), 2 reps
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for r in 1 2; do
  for v in cur $AB_VARIANTS; do
    if [ $v = cur ]; then L=""; else L=variants/libpacgpu_$v.so; fi
    echo -n "$v: "; env ${L:+PAC_LIB=$L} timeout -k 10 120 python bench.py --no-cpu --steps 3 --warmup 1 ${AB_ARGS:-} 2>&1 | grep -o '"value": [0-9.]*\|"kernels_ms": {[^}]*}' | tr '\n' ' ' || exit 1; echo
  done
done > gpurun_out/t12.log
cat gpurun_out/t12.log
