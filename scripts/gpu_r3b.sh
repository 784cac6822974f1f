#!/bin/bash
# GPU numerics of this round's fusions / kernels, then in-step A/Bs: fused stem + dual-BN backward (ResNet-50) and
# the attention backward v2 (BERT-base).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-r3b}
val() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" "$1"; }
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread \
    -k "stem or dual_bn or bn_backward_stats or conv_bn or masked_residual or tiny or resnet or bert_embeddings or attention" \
    > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for i in 1 2; do
  for cfg in "MDTF_FUSED_STEM=1 MDTF_DUAL_BWD_FUSED=1" "MDTF_FUSED_STEM=0 MDTF_DUAL_BWD_FUSED=0"; do
    env $cfg timeout -k 10 300 python bench.py --steps 20 --warmup 5 --bert 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
      || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
    echo "resnet $cfg $(val gpurun_out/bench_$TAG.json)"
  done
  for cfg in "MDTF_ATTN_BWD=v2 MDTF_BERT_EMBED=1" "MDTF_ATTN_BWD=v1 MDTF_BERT_EMBED=0"; do
    env $cfg timeout -k 10 300 python bench/bert_bench.py --steps 20 --warmup 5 > gpurun_out/bert_$TAG.json 2> gpurun_out/bert_$TAG.err \
      || { echo "bert $cfg failed"; tail -20 gpurun_out/bert_$TAG.err; exit 1; }
    echo "bert $cfg $(val gpurun_out/bert_$TAG.json)"
  done
done
