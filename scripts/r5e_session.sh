cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python bench/gemm_pp_probe.py --check > gpurun_out/ppcheck_r5e.log 2>&1; rc=$?; grep -c '"ok": true' gpurun_out/ppcheck_r5e.log; grep '"ok": false' gpurun_out/ppcheck_r5e.log | head -5; [ $rc -eq 0 ] && \
bash scripts/gpu.sh bertab r5e "MDTF_PP_FWD=act" "MDTF_PP_FWD=all MDTF_PP_DGRAD=all" 30 && \
bash scripts/gpu.sh bertab r5e2 "MDTF_PP_FWD=fused" "MDTF_PP_FWD=all MDTF_PP_DGRAD=fused" 30
