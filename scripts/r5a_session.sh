cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_r5a.log 2>&1 && tail -1 gpurun_out/bench_r5a.log | cut -c1-300 && \
bash scripts/gpu.sh prof r5a && \
timeout -k 10 400 python bench/gemm_ksweep.py > gpurun_out/ksweep_r5a.log 2>&1 && cat gpurun_out/ksweep_r5a.log | cut -c1-400
