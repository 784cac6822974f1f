#!/bin/bash
# BERT-base with the weight-gradient kernel vs the r2 conv-kernel wgrad (alternating, two passes), plus the dense GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-wgb}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "dense or ffn or bert or gemm" \
    --timeout 150 --timeout-method thread > gpurun_out/pytest_dense_$TAG.log 2>&1 \
  || { echo "pytest failed"; tail -30 gpurun_out/pytest_dense_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_dense_$TAG.log
for pass in 1 2; do
  for mode in wg none; do
    MDTF_PP_WGRAD=$mode timeout -k 10 300 python bench/bert_bench.py --steps 30 --warmup 5 > gpurun_out/bert_${mode}_${TAG}_$pass.json 2> gpurun_out/bert_${mode}_${TAG}_$pass.err \
      || { echo "bert $mode failed"; tail -20 gpurun_out/bert_${mode}_${TAG}_$pass.err; exit 1; }
    echo "$mode $pass $(tail -1 gpurun_out/bert_${mode}_${TAG}_$pass.json | cut -c1-140)"
  done
done
