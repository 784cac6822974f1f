#!/bin/bash
# Fused bias gradient in the dense weight-gradient kernel: tests, then the BERT bench A/B.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
TAG=${1:-fb1}
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_hip_graph.py -x -q -m gpu -k "wgrad or gemm or bert or dense or graph" --timeout 120 --timeout-method thread > gpurun_out/fbias_${TAG}_tests.log 2>&1 || { echo "tests rc=$?"; tail -30 gpurun_out/fbias_${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/fbias_${TAG}_tests.log
for i in 1 2; do
  for v in 1 0; do
    MDTF_FUSED_BIAS_GRAD=$v timeout -k 10 200 python bench/bert_bench.py --steps 30 --warmup 5 > gpurun_out/fb_${TAG}_$v$i.json 2> gpurun_out/fb_${TAG}_$v$i.err || { echo "bert failed"; tail -20 gpurun_out/fb_${TAG}_$v$i.err; exit 1; }
    echo "MDTF_FUSED_BIAS_GRAD=$v run $i: $(python -c "import json; d=json.load(open('gpurun_out/fb_${TAG}_$v$i.json')); print(d['value'])")"
  done
done
