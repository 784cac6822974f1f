#!/bin/bash
# GPU job: conv tests, autotune of PASSES (merged into a copy of the table), bench with the merged table,
# rocprofv3 kernel stats of a short bench.   usage: gpu_tune.sh TAG PASSES [STRIDES]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=$1; PASSES=$2; STRIDES=${3:-}
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_kernels_property.py tests/test_winograd.py -q -m gpu -k "${KF:-conv}" \
  > gpurun_out/pytest_conv_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_conv_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_conv_$TAG.log
cp mdtf/ops/conv_table.json gpurun_out/conv_table_$TAG.json
if [ -n "$PASSES" ]; then
  timeout -k 10 900 python bench/conv_autotune.py --passes $PASSES ${STRIDES:+--strides $STRIDES} --merge --reps 8 \
    --out gpurun_out/conv_table_$TAG.json --report gpurun_out/conv_autotune_$TAG.md > gpurun_out/autotune_$TAG.log 2>&1 \
    || { tail -20 gpurun_out/autotune_$TAG.log; exit 1; }
  tail -1 gpurun_out/autotune_$TAG.log
  cp gpurun_out/conv_table_$TAG.json mdtf/ops/conv_table.json
fi
timeout -k 10 400 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run \
  -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 8 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log" 2>&1 \
  || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG.log"; exit 1; }
echo done
