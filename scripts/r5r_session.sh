cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "bn or batch_norm or resnet_stage1 or fanout" > gpurun_out/pytest_r5r.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r5r.log; [ $rc -eq 0 ] && \
bash scripts/gpu.sh envab r5r "MDTF_BN_NT=1" "MDTF_BN_NT=0" 30
