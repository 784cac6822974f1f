cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "adam or momentum or optim or sgd or weight_stationary or conv3_rows or v2_8wave or dgrad or bn_backward" > gpurun_out/pytest_r5s.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r5s.log; [ $rc -eq 0 ] && \
bash scripts/gpu.sh envab r5s "MDTF_NT_EPI=1" "MDTF_NT_EPI=0" 30 && \
bash scripts/gpu.sh envab r5so "MDTF_NT_OPT=1" "MDTF_NT_OPT=0" 30 && \
bash scripts/gpu.sh bertab r5sb "MDTF_NT_OPT=1" "MDTF_NT_OPT=0" 30
