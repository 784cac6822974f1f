#!/bin/bash
# GPU job: ws kernel tests, fwd/dgrad conv autotune with the weight-stationary candidates (merged into a
# copy of the shipped table), then an A/B of bench.py with the shipped table and the new one.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-tune}
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "weight_stationary or conv" --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
cp mdtf/ops/conv_table.json gpurun_out/conv_table_$TAG.json
timeout -k 10 900 python -u bench/conv_autotune.py --passes ${PASSES:-fwd,dgrad} --merge --out gpurun_out/conv_table_$TAG.json \
    --report gpurun_out/conv_autotune_$TAG.md > gpurun_out/autotune_$TAG.log 2>&1 || { echo "autotune failed"; tail -20 gpurun_out/autotune_$TAG.log; exit 1; }
tail -1 gpurun_out/autotune_$TAG.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --bert 0 > gpurun_out/bench_${TAG}_old$i.json 2>/dev/null || exit 1
  MDTF_CONV_TABLE=gpurun_out/conv_table_$TAG.json timeout -k 10 200 python bench.py --steps 20 --warmup 5 --bert 0 \
      > gpurun_out/bench_${TAG}_new$i.json 2>/dev/null || exit 1
  python -c "import json,sys; a=json.load(open('gpurun_out/bench_${TAG}_old$i.json')); b=json.load(open('gpurun_out/bench_${TAG}_new$i.json')); print('old', a['value'], 'new', b['value'])"
done
