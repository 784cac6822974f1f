#!/bin/bash
# GPU job: kernel-only GPU time per ResNet-50 step, mdtf vs the stock PyTorch comparator (two rocprof runs each,
# 5 and 15 timed steps; the difference cancels build/warm-up/autotune).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for which in mdtf stock; do
  for s in 5 15; do
    if [ $which = mdtf ]; then prog="$R/bench.py --bert 0"; else prog="$R/bench/stock_pytorch.py"; fi
    cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/kt_${which}_$s" -o run --output-format csv \
        -- python $prog --steps $s --warmup 3 > "$R/gpurun_out/kt_${which}_$s.log" 2>&1 \
        || { echo "rocprof $which $s failed"; tail -20 "$R/gpurun_out/kt_${which}_$s.log"; exit 1; }
    cd "$R"
  done
  a=$(ls gpurun_out/kt_${which}_5/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/kt_${which}_5/run_kernel_stats.csv)
  b=$(ls gpurun_out/kt_${which}_15/*/run_kernel_stats.csv 2>/dev/null || ls gpurun_out/kt_${which}_15/run_kernel_stats.csv)
  echo "$which kernel ms/step: $(python scripts/kernel_time_diff.py $a 5 $b 15)"
done
