cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 1100 python -u bench/conv_step_tune.py --passes fwd --top 5 --budget_s 900 \
  --out gpurun_out/conv_table_step_r5aq.json --report gpurun_out/conv_step_tune_r5aq.md > gpurun_out/conv_step_tune_r5aq.log 2>&1; rc=$?; tail -4 gpurun_out/conv_step_tune_r5aq.log; exit $rc
