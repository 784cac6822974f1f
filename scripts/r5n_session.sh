cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "dual or projection_dgrad or fanout or masked_residual or wgrad_slab" > gpurun_out/pytest_r5n.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r5n.log; [ $rc -eq 0 ] && \
bash scripts/gpu.sh envab r5n "MDTF_PROJ_LATE=1" "MDTF_PROJ_LATE=0" 30
