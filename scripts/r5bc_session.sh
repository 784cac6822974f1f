# stock PyTorch-ROCm comparators on the final box, beside one mdtf run of each bench (same box, same session)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python bench/stock_pytorch.py --steps 20 --warmup 5 > gpurun_out/stock_resnet_r5bc.log 2>&1 && tail -1 gpurun_out/stock_resnet_r5bc.log | cut -c1-200 && \
timeout -k 10 400 python bench/bert_bench.py --stock --steps 20 --warmup 5 > gpurun_out/stock_bert_r5bc.log 2>&1 && tail -1 gpurun_out/stock_bert_r5bc.log | cut -c1-200 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/mdtf_r5bc.log 2>&1 && tail -1 gpurun_out/mdtf_r5bc.log | cut -c1-200
