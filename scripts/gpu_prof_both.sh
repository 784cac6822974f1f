#!/bin/bash
SKIP_BERT=${SKIP_BERT:-0}
# Kernel stats of the captured BERT-base and ResNet-50 steps (rocprofv3 --kernel-trace --stats) + summaries.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$ROOT/gpurun_out"
export TMPDIR=/tmp
TAG=${1:-pb}
[ "$SKIP_BERT" = 1 ] || bash "$ROOT/scripts/gpu_bert_prof.sh" $TAG > "$ROOT/gpurun_out/bert_prof_$TAG.txt" || exit 1
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_resnet_$TAG" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 5 --warmup 3 --bert 0 > "$ROOT/gpurun_out/prof_resnet_$TAG.log" 2>&1 \
  || { echo "resnet prof failed"; tail -20 "$ROOT/gpurun_out/prof_resnet_$TAG.log"; exit 1; }
python3 "$ROOT/scripts/step_breakdown.py" "$ROOT/gpurun_out/prof_resnet_$TAG/run_kernel_trace.csv" > "$ROOT/gpurun_out/resnet_steps_$TAG.txt"
head -12 "$ROOT/gpurun_out/resnet_steps_$TAG.txt"
python3 "$ROOT/scripts/prof_summary.py" "$ROOT/gpurun_out/prof_resnet_$TAG/run_kernel_stats.csv" 8 > "$ROOT/gpurun_out/resnet_prof_$TAG.txt"
