cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash scripts/gpu.sh tests r5be && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" && \
timeout -k 10 300 python bench.py > gpurun_out/bench_default_r5be.log 2>&1 && tail -1 gpurun_out/bench_default_r5be.log | cut -c1-300
