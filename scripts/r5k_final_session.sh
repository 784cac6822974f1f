cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash scripts/gpu.sh tests r5k && \
bash scripts/gpu.sh bench r5k --steps 30 --warmup 5 && \
bash scripts/gpu.sh prof r5k > /dev/null && echo "prof ok"
