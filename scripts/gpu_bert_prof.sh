#!/bin/bash
# rocprofv3 kernel stats of the captured BERT-base step (env passed through: e.g. MDTF_PP_WGRAD=wg).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$ROOT/gpurun_out"
export TMPDIR=/tmp
TAG=${1:-bp}
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_bert_$TAG" -o run --output-format csv \
    -- python3 "$ROOT/bench/bert_bench.py" --steps 5 --warmup 3 > "$ROOT/gpurun_out/prof_bert_$TAG.log" 2>&1 \
  || { echo "bert prof failed"; tail -20 "$ROOT/gpurun_out/prof_bert_$TAG.log"; exit 1; }
python3 "$ROOT/scripts/prof_summary.py" "$ROOT/gpurun_out/prof_bert_$TAG/run_kernel_stats.csv" 8 > "$ROOT/gpurun_out/bert_summary_$TAG.txt"
head -30 "$ROOT/gpurun_out/bert_summary_$TAG.txt"
