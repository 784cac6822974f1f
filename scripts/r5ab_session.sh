cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
bash scripts/gpu.sh envab r5abf "MDTF_CONV_TABLE=profiles/conv_table_cand_r5aa_fwd.json" "MDTF_CONV_TABLE=mdtf/ops/conv_table.json" 30 && \
bash scripts/gpu.sh envab r5abd "MDTF_CONV_TABLE=profiles/conv_table_cand_r5aa_dgrad.json" "MDTF_CONV_TABLE=mdtf/ops/conv_table.json" 30
