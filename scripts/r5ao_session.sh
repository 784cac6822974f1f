cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash scripts/gpu.sh tests r5ao && \
bash scripts/gpu.sh bertab r5ao1 "MDTF_PP_FWD=act" "MDTF_PP_FWD=fused" 30 && \
bash scripts/gpu.sh bertab r5ao2 "MDTF_PP_DGRAD=fused" "MDTF_PP_DGRAD=all" 30
