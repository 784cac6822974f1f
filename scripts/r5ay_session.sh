cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 1100 python -u bench/conv_step_tune.py --passes dgrad --rank_epilogue --top 4 --budget_s 900 \
  --out gpurun_out/conv_table_step_r5ay.json --report gpurun_out/conv_step_tune_r5ay.md > gpurun_out/conv_step_tune_r5ay.log 2>&1; rc=$?; tail -6 gpurun_out/conv_step_tune_r5ay.log; exit $rc
