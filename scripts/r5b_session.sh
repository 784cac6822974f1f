cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "attention or pooled" > gpurun_out/pytest_r5b.log 2>&1; rc=$?; tail -25 gpurun_out/pytest_r5b.log; [ $rc -eq 0 ] && \
timeout -k 10 200 python bench/attn_probe.py > gpurun_out/attn_probe_r5b.log 2>&1 && tail -3 gpurun_out/attn_probe_r5b.log
