#!/bin/bash
# Weight-gradient kernel GPU tests, then the config sweep on the BERT-base shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-wgt}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "gemm_wg" --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_wg_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_wg_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_wg_$TAG.log
SHAPES=${SHAPES:-qkv,ffn_in,ffn_out,attn_out} bash scripts/gpu_wg.sh $TAG
