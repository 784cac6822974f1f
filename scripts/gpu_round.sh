#!/bin/bash
# GPU job: GPU test suite, smoke(), 1-GPU bench, rocprofv3 kernel stats. Stops at the first failing GPU step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-run}
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
    || { echo "smoke failed"; tail -30 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
    || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
if [ -n "$PROF" ]; then
  cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run \
      --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1
  echo "prof exit $?"
fi
