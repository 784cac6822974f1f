#!/bin/bash
# Fused stem / dual-BN backward: GPU numerics tests, in-step A/B of the fusions, then the in-step conv tuner.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-r3b}
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -v -m gpu --timeout 120 --timeout-method thread \
    -k "stem or dual_bn or bn_backward_stats or conv_bn or masked_residual or tiny or resnet or bert_embeddings" > gpurun_out/pytest_$TAG.log 2>&1 \
  || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for i in 1 2; do
  for cfg in "MDTF_FUSED_STEM=1" "MDTF_FUSED_STEM=0 MDTF_DUAL_BWD_FUSED=0"; do
    env $cfg timeout -k 10 300 python bench.py --steps 20 --warmup 5 --bert 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
      || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
    echo "$cfg $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" gpurun_out/bench_$TAG.json)"
  done
done
if [ "${TUNE:-1}" = 1 ]; then
  timeout -k 10 900 python -u bench/conv_step_tune.py --budget_s ${BUDGET:-540} --out gpurun_out/conv_table_$TAG.json \
      --report gpurun_out/conv_step_tune_$TAG.md > gpurun_out/step_tune_$TAG.log 2>&1 \
    || { echo "step tune failed"; tail -30 gpurun_out/step_tune_$TAG.log; exit 1; }
  tail -2 gpurun_out/step_tune_$TAG.log
  MDTF_CONV_TABLE=gpurun_out/conv_table_$TAG.json timeout -k 10 300 python bench.py --steps 20 --warmup 5 --bert 0 \
      > gpurun_out/bench_${TAG}_tuned.json 2> gpurun_out/bench_${TAG}_tuned.err \
    || { echo "bench tuned failed"; tail -20 gpurun_out/bench_${TAG}_tuned.err; exit 1; }
  echo "tuned $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" gpurun_out/bench_${TAG}_tuned.json)"
fi
