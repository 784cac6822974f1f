#!/bin/bash
# GPU job: hipGraph step tests, then ResNet-50 / BERT-base benches eager vs graph.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-g}
timeout -k 10 300 python -u -m pytest tests/test_hip_graph.py tests/test_kernels_gpu.py -x -v -m gpu --timeout 120 \
    --timeout-method thread -k "graph or optimizer or layernorm or attention" > gpurun_out/pytest_$TAG.log 2>&1 \
    || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -3 gpurun_out/pytest_$TAG.log
for g in 0 1; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --hip_graph $g > gpurun_out/bench_${TAG}_g$g.json \
      2> gpurun_out/bench_${TAG}_g$g.err || { echo "bench g=$g failed"; tail -30 gpurun_out/bench_${TAG}_g$g.err; exit 1; }
  cat gpurun_out/bench_${TAG}_g$g.json
done
for g in 0 1; do
  timeout -k 10 200 python bench/bert_bench.py --steps 20 --warmup 5 --hip_graph $g > gpurun_out/bert_${TAG}_g$g.json \
      2> gpurun_out/bert_${TAG}_g$g.err || { echo "bert g=$g failed"; tail -30 gpurun_out/bert_${TAG}_g$g.err; exit 1; }
  cat gpurun_out/bert_${TAG}_g$g.json
done
