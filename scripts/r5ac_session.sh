cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 1100 python -u bench/conv_step_tune.py --passes fwd,dgrad --budget_s 780 --out gpurun_out/conv_table_step_r5ac.json --report gpurun_out/conv_step_tune_r5ac.md > gpurun_out/step_tune_r5ac.log 2>&1; rc=$?; tail -15 gpurun_out/step_tune_r5ac.log; exit $rc
