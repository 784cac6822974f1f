cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python -u bench/gemm_pp_probe.py --check > gpurun_out/pp_check_r5af.log 2>&1; rc=$?; grep -c '"ok": true' gpurun_out/pp_check_r5af.log; grep '"ok": false' gpurun_out/pp_check_r5af.log | head -3; [ $rc -eq 0 ] && \
timeout -k 10 120 python -u bench/act_dgrad_probe.py && MDTF_PP_PRE_LDS=0 timeout -k 10 120 python -u bench/act_dgrad_probe.py && \
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "gemm_pp or dense or ffn or bert" > gpurun_out/pytest_r5af.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r5af.log; [ $rc -eq 0 ] && \
bash scripts/gpu.sh bertab r5af "MDTF_ACT_DGRAD=core" "MDTF_ACT_DGRAD=conv" 30
