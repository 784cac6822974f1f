cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "dgrad or conv_hip or resid or bn_backward_stats" > gpurun_out/pytest_r5f.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r5f.log; [ $rc -eq 0 ] && \
bash scripts/gpu.sh envab r5f "MDTF_DGRAD_PREFETCH=1" "MDTF_DGRAD_PREFETCH=0" 30
