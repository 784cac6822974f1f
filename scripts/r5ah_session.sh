cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "wgrad or zero_class or dgrad" > gpurun_out/pytest_r5ah.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r5ah.log; [ $rc -eq 0 ] && \
bash scripts/gpu.sh envab r5ah "MDTF_SLAB_NT=1" "MDTF_SLAB_NT=0" 30
