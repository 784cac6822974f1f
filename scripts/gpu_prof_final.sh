#!/bin/bash
# GPU job: rocprofv3 kernel stats of the final ResNet-50 and BERT-base steps.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_final_resnet" -o run --output-format csv \
    -- python "$R/bench.py" --steps 5 --warmup 3 --bert 0 > "$R/gpurun_out/prof_final_resnet.log" 2>&1 || { echo "resnet prof failed"; exit 1; }
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_final_bert" -o run --output-format csv \
    -- python "$R/bench/bert_bench.py" --steps 5 --warmup 3 > "$R/gpurun_out/prof_final_bert.log" 2>&1 || { echo "bert prof failed"; exit 1; }
echo done
