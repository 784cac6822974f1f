cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "xent or bert or decoder or softmax or dense" > gpurun_out/pytest_r5aj.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r5aj.log; [ $rc -eq 0 ] && \
bash scripts/gpu.sh bertab r5aj "MDTF_DEC_SPLIT=8" "MDTF_DEC_SPLIT=0" 30 && \
timeout -k 10 1000 python -u bench/conv_step_tune.py --passes dgrad --rank_epilogue --budget_s 780 \
  --out gpurun_out/conv_table_step_r5aj.json --report gpurun_out/conv_step_tune_r5aj.md > gpurun_out/conv_step_tune_r5aj.log 2>&1; rc=$?; tail -5 gpurun_out/conv_step_tune_r5aj.log; exit $rc
