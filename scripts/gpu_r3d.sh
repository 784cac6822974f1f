#!/bin/bash
# In-step conv tile tuning of the ResNet-50 step, then bench.py with the tuned table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-r3d}
timeout -k 10 900 python -u bench/conv_step_tune.py --budget_s ${BUDGET:-600} --top ${TOP:-3} --out gpurun_out/conv_table_$TAG.json \
    --report gpurun_out/conv_step_tune_$TAG.md > gpurun_out/step_tune_$TAG.log 2>&1 \
  || { echo "step tune failed"; tail -30 gpurun_out/step_tune_$TAG.log; exit 1; }
tail -2 gpurun_out/step_tune_$TAG.log
MDTF_CONV_TABLE=gpurun_out/conv_table_$TAG.json timeout -k 10 300 python bench.py --steps 20 --warmup 5 --bert 0 \
    > gpurun_out/bench_${TAG}_tuned.json 2> gpurun_out/bench_${TAG}_tuned.err \
  || { echo "bench tuned failed"; tail -20 gpurun_out/bench_${TAG}_tuned.err; exit 1; }
echo "tuned $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" gpurun_out/bench_${TAG}_tuned.json)"
