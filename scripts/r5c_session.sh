cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv_pp or gemm_pp or pp_" > gpurun_out/pytest_r5c.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r5c.log; [ $rc -eq 0 ] && \
timeout -k 10 300 python bench/gemm_pp_probe.py --check > gpurun_out/ppcheck_r5c.log 2>&1; rc=$?; grep -c '"ok": true' gpurun_out/ppcheck_r5c.log; grep '"ok": false' gpurun_out/ppcheck_r5c.log | head -5; [ $rc -eq 0 ] && \
timeout -k 10 400 python bench/gemm_ksweep.py --N 3072,768 --K 64,256,768,3072 --tiles 0,4,5 > gpurun_out/ksweep_r5c.log 2>&1 && cut -c1-300 gpurun_out/ksweep_r5c.log && \
timeout -k 10 600 python bench/conv_pp_probe.py --out gpurun_out/conv_pp_probe_r5c.jsonl > gpurun_out/conv_pp_probe_r5c.log 2>&1; tail -40 gpurun_out/conv_pp_probe_r5c.log
