#!/bin/bash
# GPU job: conv kernel tests -> per-shape autotune -> bench with the tuned table -> profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-conv}
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu_$TAG.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench/conv_autotune.py --out gpurun_out/conv_table.json --report gpurun_out/conv_autotune.md > gpurun_out/autotune_$TAG.log 2>&1 &&
cp gpurun_out/conv_table.json mdtf/ops/conv_table.json &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 5 --warmup 3 > gpurun_out/prof_$TAG.log 2>&1
echo "exit $?"
