cd $GRAFT_REPO_ROOT
for v in "$@"; do
  echo -n "$v: "; PAC_LIB=variants/libpacgpu_$v.so timeout -k 10 120 python bench.py --no-cpu --steps 3 --warmup 1 ${AB_ARGS:---config 1} 2>&1 | grep -o '"kernels_ms": {[^}]*}' || exit 1
done
