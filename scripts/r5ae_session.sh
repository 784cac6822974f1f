cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "wgrad" > gpurun_out/pytest_r5ae.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r5ae.log; [ $rc -eq 0 ] && \
bash scripts/gpu.sh envab r5ae "MDTF_SLAB_LANES=4" "MDTF_SLAB_LANES=1" 30
