#!/bin/bash
# GPU tests selected by -k, then two BERT-base bench runs.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
TAG=${1:-bc}; KEXPR=${2:-bert}
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_hip_graph.py -x -q -m gpu -k "$KEXPR" --timeout 120 --timeout-method thread > gpurun_out/bc_${TAG}_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/bc_${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/bc_${TAG}_tests.log
for i in 1 2; do
  timeout -k 10 200 python bench/bert_bench.py --steps 30 --warmup 5 > gpurun_out/bc_${TAG}_$i.json 2> gpurun_out/bc_${TAG}_$i.err || { echo "bert failed"; tail -20 gpurun_out/bc_${TAG}_$i.err; exit 1; }
  echo "bert run $i: $(python -c "import json; d=json.load(open('gpurun_out/bc_${TAG}_$i.json')); print(d['value'])")"
done
