cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv_pp" > gpurun_out/pytest_r5g.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r5g.log; [ $rc -eq 0 ] && \
timeout -k 10 600 python bench/conv_pp_probe.py --out gpurun_out/conv_pp_probe_r5g.jsonl > gpurun_out/conv_pp_probe_r5g.log 2>&1; tail -40 gpurun_out/conv_pp_probe_r5g.log
