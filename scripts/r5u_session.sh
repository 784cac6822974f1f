cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "gemm_wg or wgrad_into or bert" > gpurun_out/pytest_r5u.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r5u.log; [ $rc -eq 0 ] && \
bash scripts/gpu.sh bertab r5u "MDTF_WG_SK=1" "MDTF_WG_SK=0" 30
