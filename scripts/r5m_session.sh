cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "dual or projection_dgrad or fanout or masked_residual or resnet_stage1 or resnet_train or conv3_rows" > gpurun_out/pytest_r5m.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r5m.log; [ $rc -eq 0 ] && \
bash scripts/gpu.sh envab r5m "MDTF_DUAL_DGRAD=1" "MDTF_DUAL_DGRAD=0" 30 && \
bash scripts/gpu.sh envab r5l "MDTF_SLAB_GROUPS=1" "MDTF_SLAB_GROUPS=0" 30
