cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "xent or bert or decoder" > gpurun_out/pytest_r5al.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r5al.log; [ $rc -eq 0 ] && \
bash scripts/gpu.sh bertab r5al "MDTF_DEC_SPLIT=8" "MDTF_DEC_SPLIT=0" 30 && \
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_bert_r5al -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench/bert_bench.py --steps 5 --warmup 3) > gpurun_out/prof_bert_r5al.log 2>&1 && \
python scripts/step_breakdown.py gpurun_out/prof_bert_r5al --calls > gpurun_out/summary_bert_r5al.txt 2>&1; head -12 gpurun_out/summary_bert_r5al.txt; grep -n "xent\|colsum\|Cijk_Ailk_Bljk_BBS_BH_Bias_HA_S_SAV_UserArgs_MT128x96\|bmm\|MT.*x.*x" gpurun_out/summary_bert_r5al.txt | sed -n 1,12p
