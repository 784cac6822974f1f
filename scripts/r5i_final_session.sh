cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash scripts/gpu.sh tests r5i && \
bash scripts/gpu.sh bench r5i --steps 30 --warmup 5 && \
bash scripts/gpu.sh prof r5i > /dev/null && echo "prof ok"
