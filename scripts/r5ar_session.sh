cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 1100 python -u bench/bert_wg_tune.py --act --budget_s 900 --report gpurun_out/bert_act_tune_r5ar.md > gpurun_out/bert_act_tune_r5ar.log 2>&1; rc=$?; tail -4 gpurun_out/bert_act_tune_r5ar.log; exit $rc
