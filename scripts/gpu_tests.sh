#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-t}
timeout -k 10 900 python -m pytest tests -q -m gpu > gpurun_out/pytest_gpu_$TAG.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu_$TAG.log
tail -5 gpurun_out/pytest_gpu_$TAG.log
