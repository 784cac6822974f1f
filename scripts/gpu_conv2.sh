#!/bin/bash
# GPU job: conv kernel tests (v1 + v2) then fwd/dgrad autotune incl. v2 tiles (table to gpurun_out only)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-c2}
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -q -m gpu -k "conv" > gpurun_out/pytest_conv_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_conv_$TAG.log
tail -3 gpurun_out/pytest_conv_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench/conv_autotune.py --passes ${PASSES:-fwd,dgrad} --reps 8 --out gpurun_out/conv_table_$TAG.json --report gpurun_out/conv_autotune_$TAG.md > gpurun_out/autotune_$TAG.log 2>&1
echo "autotune rc=$?"
tail -2 gpurun_out/autotune_$TAG.log
