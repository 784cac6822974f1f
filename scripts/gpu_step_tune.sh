#!/bin/bash
# In-step conv tile tuning of the ResNet-50 step, then bench.py with the default and the tuned table.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-st1}
timeout -k 10 1000 python -u bench/conv_step_tune.py --budget_s ${BUDGET:-600} ${TUNE_ARGS} --out gpurun_out/conv_table_$TAG.json \
    --report gpurun_out/conv_step_tune_$TAG.md > gpurun_out/step_tune_$TAG.log 2>&1 \
  || { echo "step tune failed"; tail -30 gpurun_out/step_tune_$TAG.log; exit 1; }
tail -3 gpurun_out/step_tune_$TAG.log
for cfg in default tuned; do
  if [ $cfg = tuned ]; then export MDTF_CONV_TABLE=gpurun_out/conv_table_$TAG.json; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --bert 0 > gpurun_out/bench_${TAG}_$cfg.json 2> gpurun_out/bench_${TAG}_$cfg.err \
    || { echo "bench $cfg failed"; tail -20 gpurun_out/bench_${TAG}_$cfg.err; exit 1; }
  echo "$cfg $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" gpurun_out/bench_${TAG}_$cfg.json)"
done
