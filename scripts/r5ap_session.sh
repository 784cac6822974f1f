cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 1100 python -u bench/bert_wg_tune.py --budget_s 900 --report gpurun_out/bert_wg_tune_r5ap.md > gpurun_out/bert_wg_tune_r5ap.log 2>&1; rc=$?; tail -6 gpurun_out/bert_wg_tune_r5ap.log; exit $rc
