cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "ws or weight_stationary or dgrad or dual or fanout or projection" > gpurun_out/pytest_r5an.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r5an.log; [ $rc -eq 0 ] && \
bash scripts/gpu.sh envab r5an "MDTF_WS_EPF=1" "MDTF_WS_EPF=0" 30
