cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash scripts/gpu.sh tests r5g && \
bash scripts/gpu.sh bench r5g --steps 30 --warmup 5 && \
bash scripts/gpu.sh prof r5g > /dev/null && echo "prof ok"
