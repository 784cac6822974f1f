cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash scripts/gpu.sh bench r5f --steps 30 --warmup 5 && \
bash scripts/gpu.sh prof r5f > /dev/null && echo "prof ok" && \
bash scripts/gpu.sh pmc r5f && echo "pmc ok"
