cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "layernorm or ln_" > gpurun_out/pytest_r5av.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r5av.log; [ $rc -eq 0 ] && \
bash scripts/gpu.sh bertab r5av1 "MDTF_LN_BWD_RPB=8" "MDTF_LN_BWD_RPB=16" 30 && \
bash scripts/gpu.sh bertab r5av2 "MDTF_LN_BWD_RPB=32" "MDTF_LN_BWD_RPB=16" 30
