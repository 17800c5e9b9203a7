cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -x -v --timeout 200 --timeout-method thread -k schedules > gpurun_out/t_sched.log 2>&1; tail -6 gpurun_out/t_sched.log
