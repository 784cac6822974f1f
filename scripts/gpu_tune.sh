#!/bin/bash
# GPU job: conv kernel tests (v2 + 8-wave tiles), then the ResNet-50 conv autotune (report + table under gpurun_out/).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-tune}
PASSES=${PASSES:-fwd,dgrad,wgrad}
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread \
    -k "conv" > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 600 python -u bench/conv_autotune.py --passes $PASSES --out gpurun_out/conv_table_$TAG.json \
    --report gpurun_out/conv_autotune_$TAG.md > gpurun_out/tune_$TAG.log 2>&1 \
    || { echo "autotune failed"; tail -30 gpurun_out/tune_$TAG.log; exit 1; }
tail -1 gpurun_out/tune_$TAG.log
