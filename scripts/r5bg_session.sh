cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "embed or bert" > gpurun_out/pytest_r5bg.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r5bg.log; [ $rc -eq 0 ] && \
bash scripts/gpu.sh bertab r5bg "MDTF_POS_BCAST=1" "MDTF_POS_BCAST=0" 30
