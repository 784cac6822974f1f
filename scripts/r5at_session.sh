cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash scripts/gpu.sh rehearse2 r5at && \
MDTF_DIST_BACKEND=gloo timeout -k 10 400 python bench/bert_bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/rehearse2_bert_r5at.json 2> gpurun_out/rehearse2_bert_r5at.err && tail -1 gpurun_out/rehearse2_bert_r5at.json | cut -c1-300 && \
MDTF_DIST_BACKEND=gloo timeout -k 10 400 python bench/bert_bench.py --gpus 2 --steps 5 --warmup 2 --mode sharded --comm_dtype bf16 > gpurun_out/rehearse2s_bert_r5at.json 2> gpurun_out/rehearse2s_bert_r5at.err && tail -1 gpurun_out/rehearse2s_bert_r5at.json | cut -c1-300
