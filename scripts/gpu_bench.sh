#!/bin/bash
# GPU job: kernel tests + native bench + rocprof stats (short).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu_$TAG.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- python bench.py --steps 5 --warmup 3 > gpurun_out/prof_$TAG.log 2>&1
echo "exit $?"
