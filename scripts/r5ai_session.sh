cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 240 ./bench/mfma_loop_probe 256 5 > gpurun_out/mfma_loop_probe_r5ai.jsonl 2>&1; rc=$?; cat gpurun_out/mfma_loop_probe_r5ai.jsonl; [ $rc -eq 0 ] && \
timeout -k 10 300 python -u bench/mlm_decoder_probe.py > gpurun_out/mlm_decoder_probe_r5ai.jsonl 2>&1; rc=$?; tail -3 gpurun_out/mlm_decoder_probe_r5ai.jsonl; exit $rc
