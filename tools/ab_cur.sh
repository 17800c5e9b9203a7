# scratch A/B driver of the current experiment (gpurun -- 'bash tools/ab_cur.sh'):
# variants/libpacgpu_<name>.so built by tools/build_variant.py / tools/build_rev.sh
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
AB_ARGS="--config 2" bash tools/ab_bench.sh base eint base eint || exit 1
