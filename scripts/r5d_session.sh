cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python bench/gemm_pp_probe.py --check > gpurun_out/ppcheck_r5d.log 2>&1; rc=$?; grep -c '"ok": true' gpurun_out/ppcheck_r5d.log; grep '"ok": false' gpurun_out/ppcheck_r5d.log | head -5; [ $rc -eq 0 ] && \
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "pp or dense or bert" > gpurun_out/pytest_r5d.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r5d.log; [ $rc -eq 0 ] && \
timeout -k 10 400 python bench/gemm_ksweep.py --N 3072,768 --K 64,256,768,3072 --tiles 0,4,5 > gpurun_out/ksweep_r5d.log 2>&1 && cut -c1-300 gpurun_out/ksweep_r5d.log && \
timeout -k 10 400 python bench/gemm_pp_probe.py --shapes qkv,attn_out,ffn_in,ffn_out,dg_qkv,dg_ffn_in,dg_ffn_out > gpurun_out/pp_probe_r5d.log 2>&1; cut -c1-600 gpurun_out/pp_probe_r5d.log
