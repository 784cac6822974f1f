cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash scripts/gpu.sh envab r5ad "MDTF_CONV_TABLE=profiles/conv_table_cand_r5ac.json" "MDTF_CONV_TABLE=mdtf/ops/conv_table.json" 30
