cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "xent or decoder" > gpurun_out/pytest_r5am.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r5am.log; [ $rc -eq 0 ] && \
for i in 1 2 3; do timeout -k 10 300 python bench/bert_bench.py --steps 30 --warmup 5 > gpurun_out/bert_r5am_$i.log 2>&1 || exit 1; tail -1 gpurun_out/bert_r5am_$i.log | cut -c1-160; done && \
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_bert_r5am -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench/bert_bench.py --steps 5 --warmup 3) > gpurun_out/prof_bert_r5am.log 2>&1 && \
python scripts/step_breakdown.py gpurun_out/prof_bert_r5am --calls > gpurun_out/summary_bert_r5am.txt 2>&1; grep -n "xent\|colsum" gpurun_out/summary_bert_r5am.txt | head -5; \
timeout -k 10 1100 python -u bench/conv_step_tune.py --passes wgrad --budget_s 900 \
  --out gpurun_out/conv_table_step_r5am.json --report gpurun_out/conv_step_tune_r5am.md > gpurun_out/conv_step_tune_r5am.log 2>&1; rc=$?; tail -4 gpurun_out/conv_step_tune_r5am.log; exit $rc
