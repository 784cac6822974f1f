cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "optimizer or adam or bn or stem or pool" > gpurun_out/pytest_r5y.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r5y.log; [ $rc -eq 0 ] && \
bash scripts/gpu.sh bertab r5y "MDTF_ADAM_CHUNK=1" "MDTF_ADAM_CHUNK=0" 30
