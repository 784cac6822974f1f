cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 1100 python bench/conv_autotune.py --passes fwd,dgrad --graph --reps 10 --step_epilogues --out gpurun_out/conv_table_fd_r5aa.json --report gpurun_out/conv_autotune_fd_r5aa.md > gpurun_out/autotune_fd_r5aa.log 2>&1; rc=$?; tail -4 gpurun_out/autotune_fd_r5aa.log; exit $rc
