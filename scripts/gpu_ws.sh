#!/bin/bash
# GPU job: weight-stationary conv kernel tests + shape probe vs the current conv table choices.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-ws}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k weight_stationary --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 400 python -u bench/conv_ws_probe.py --out gpurun_out/probe_$TAG.json > gpurun_out/probe_$TAG.log 2>&1 \
    || { echo "probe failed"; tail -30 gpurun_out/probe_$TAG.log; exit 1; }
grep BEST gpurun_out/probe_$TAG.log
