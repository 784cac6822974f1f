cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash scripts/gpu.sh tests r5h && \
bash scripts/gpu.sh bench r5h --steps 30 --warmup 5 && \
bash scripts/gpu.sh prof r5h > /dev/null && echo "prof ok"
