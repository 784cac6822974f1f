#!/bin/bash
# LayerNorm kernels: GPU tests, then the BERT-base kernel stats (ln_fwd / ln_bwd per call) and bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-ln}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "layernorm or bert" --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_ln_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_ln_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_ln_$TAG.log
bash scripts/gpu_bert_prof.sh $TAG | grep -E "total|ln_|reduce_partials"
timeout -k 10 300 python bench/bert_bench.py --steps 30 --warmup 5 > gpurun_out/bert_$TAG.json 2> gpurun_out/bert_$TAG.err \
  || { echo "bert failed"; tail -10 gpurun_out/bert_$TAG.err; exit 1; }
tail -1 gpurun_out/bert_$TAG.json | cut -c1-150
