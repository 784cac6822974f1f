cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "conv3_rows or stem or conv_pp or weight_stationary" > gpurun_out/pytest_r5j.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r5j.log; [ $rc -eq 0 ] && \
timeout -k 10 300 python -u bench/conv_rows_probe.py > gpurun_out/conv_rows_probe_r5j.jsonl 2>&1; rc=$?; tail -2 gpurun_out/conv_rows_probe_r5j.jsonl; [ $rc -eq 0 ] && \
bash scripts/gpu.sh envab r5j "MDTF_CONV_ROWS=1" "MDTF_CONV_ROWS=0" 30 && \
bash scripts/gpu.sh envab r5jt "MDTF_CONV_TABLE=profiles/conv_table_cand_r5i.json" "MDTF_CONV_TABLE=mdtf/ops/conv_table.json" 30
