cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_bert_r5ak -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench/bert_bench.py --steps 5 --warmup 3) > gpurun_out/prof_bert_r5ak.log 2>&1 && \
python scripts/step_breakdown.py gpurun_out/prof_bert_r5ak --calls > gpurun_out/summary_bert_r5ak.txt 2>&1; head -45 gpurun_out/summary_bert_r5ak.txt
