cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && ALT=$GRAFT_REPO_ROOT/mdtf/csrc/build/alt/libmdtf_kernels_head.so && \
timeout -k 10 120 python bench/dgrad_conflict_probe.py > gpurun_out/dgrad_epi_new_r5az.log 2>&1 && \
MDTF_KERNELS_LIB=$ALT timeout -k 10 120 python bench/dgrad_conflict_probe.py > gpurun_out/dgrad_epi_head_r5az.log 2>&1 && \
paste gpurun_out/dgrad_epi_new_r5az.log gpurun_out/dgrad_epi_head_r5az.log | grep tile && \
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 200 --timeout-method thread -k "dgrad or fanout or accumulate or conv" > gpurun_out/pytest_r5az.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_r5az.log; [ $rc -eq 0 ] && \
bash scripts/gpu.sh envab r5az "MDTF_FD_NOTE=new" "MDTF_KERNELS_LIB=$ALT" 30
