cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "ws or stem or dense_dgrad or bn_backward_stats or resid" > gpurun_out/pytest_r5i.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_r5i.log; [ $rc -eq 0 ] && \
bash scripts/gpu.sh bertab r5i "MDTF_ACT_DGRAD=conv" "MDTF_ACT_DGRAD=core" 30 && \
bash scripts/r5h_session.sh
