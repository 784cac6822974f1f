cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/pmc_dgc_r5aw -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench/dgrad_conflict_probe.py) > gpurun_out/pmc_dgc_r5aw.log 2>&1 && \
python scripts/dgrad_conflict_summary.py gpurun_out/pmc_dgc_r5aw > gpurun_out/dgrad_conflicts_r5aw.txt 2>&1; cat gpurun_out/dgrad_conflicts_r5aw.txt
