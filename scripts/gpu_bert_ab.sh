#!/bin/bash
# BERT-base A/B of the dense-engine policies, alternating, on one box; then the dense GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-ab}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "dense or ffn or bert or gemm" \
    --timeout 150 --timeout-method thread > gpurun_out/pytest_dense_$TAG.log 2>&1 \
  || { echo "pytest failed"; tail -30 gpurun_out/pytest_dense_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_dense_$TAG.log
for i in 1 2; do
  for cfg in "MDTF_DENSE=pp" "MDTF_DENSE=legacy" "MDTF_DENSE=pp MDTF_PP_FWD=all" "MDTF_DENSE=pp MDTF_PP_WGRAD=all"; do
    env $cfg timeout -k 10 300 python bench/bert_bench.py --steps 20 --warmup 5 > gpurun_out/bert_ab_$TAG.json 2> gpurun_out/bert_ab_$TAG.err \
        || { echo "bert $cfg failed"; tail -20 gpurun_out/bert_ab_$TAG.err; exit 1; }
    echo "$cfg $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" gpurun_out/bert_ab_$TAG.json)"
  done
done
