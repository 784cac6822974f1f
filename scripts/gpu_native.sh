#!/bin/bash
# GPU job: kernel numerics tests, native bench, rocprof kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_native.json 2> gpurun_out/bench_native.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_native -o run --output-format csv -- python bench.py --steps 5 --warmup 3 > gpurun_out/prof_native.log 2>&1
echo "exit $?"
