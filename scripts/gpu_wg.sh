#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-wg}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread \
    -k "wgrad or gemm" > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python bench/gemm_micro.py > gpurun_out/gemm_$TAG.md 2>&1 || { echo "gemm micro failed"; tail -20 gpurun_out/gemm_$TAG.md; exit 1; }
cat gpurun_out/gemm_$TAG.md
timeout -k 10 600 python -u bench/conv_autotune.py --passes wgrad --out gpurun_out/conv_table_$TAG.json \
    --report gpurun_out/conv_autotune_$TAG.md > gpurun_out/tune_$TAG.log 2>&1 || { echo "autotune failed"; tail -30 gpurun_out/tune_$TAG.log; exit 1; }
tail -1 gpurun_out/tune_$TAG.log
