cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "bn or resnet or dgrad or fanout or early" > gpurun_out/pytest_r5bb.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r5bb.log; [ $rc -eq 0 ] && \
bash scripts/gpu.sh envab r5bb "MDTF_BN_EARLY_FIN=1" "MDTF_BN_EARLY_FIN=0" 30
