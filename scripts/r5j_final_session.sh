cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash scripts/gpu.sh tests r5j && \
bash scripts/gpu.sh bench r5j --steps 30 --warmup 5 && \
bash scripts/gpu.sh prof r5j > /dev/null && echo "prof ok"
