#!/bin/bash
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
TAG=${1:-x1}
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "xent or bert" --timeout 120 --timeout-method thread > gpurun_out/xent_${TAG}_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/xent_${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/xent_${TAG}_tests.log
for i in 1 2; do
  timeout -k 10 200 python bench/bert_bench.py --steps 30 --warmup 5 > gpurun_out/xb_${TAG}_$i.json 2> gpurun_out/xb_${TAG}_$i.err || { echo "bert failed"; tail -20 gpurun_out/xb_${TAG}_$i.err; exit 1; }
  echo "bert run $i: $(python -c "import json; d=json.load(open('gpurun_out/xb_${TAG}_$i.json')); print(d['value'])")"
done
