cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
AB_ENVS="PAC_SIDE_LDS_PAD=0 PAC_SIDE_LDS_PAD=8192 PAC_SIDE_LDS_PAD=22000 PAC_SIDE_LDS_PAD=48000" bash tools/ab_env.sh > gpurun_out/t13.log 2>&1
cat gpurun_out/t13.log
