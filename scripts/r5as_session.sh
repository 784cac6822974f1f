cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash scripts/gpu.sh bertab r5as "MDTF_DENSE_WGRAD_STREAM=1" "MDTF_DENSE_WGRAD_STREAM=0" 30
