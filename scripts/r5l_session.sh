cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "wgrad" > gpurun_out/pytest_r5l.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r5l.log; [ $rc -eq 0 ] && \
bash scripts/gpu.sh envab r5l "MDTF_SLAB_GROUPS=1" "MDTF_SLAB_GROUPS=0" 30
