cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "layernorm or ln_ or bert" > gpurun_out/pytest_r5bd.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r5bd.log; [ $rc -eq 0 ] && \
bash scripts/gpu.sh bertab r5bd "MDTF_LN_NT=1" "MDTF_LN_NT=0" 30
