# tail timing-only variants (garbage bytes): no lines loop / no BitAlloc rounds, vs the current build
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for v in cur tnolines tnoba; do
  if [ $v = cur ]; then L=""; else L=variants/libpacgpu_$v.so; fi
  echo -n "$v: "; env ${L:+PAC_LIB=$L} timeout -k 10 120 python bench.py --no-cpu --steps 3 --warmup 1 2>&1 | grep -o '"value": [0-9.]*\|"kernels_ms": {[^}]*}' | tr '\n' ' '; echo
done > gpurun_out/t7.log
cat gpurun_out/t7.log
