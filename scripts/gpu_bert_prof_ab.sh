#!/bin/bash
# rocprofv3 kernel stats of the graph-captured BERT-base step under two dense-engine settings.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$ROOT/gpurun_out"
export TMPDIR=/tmp
TAG=${1:-bpa}
cd /tmp
for mode in pp legacy; do
  MDTF_DENSE=$mode timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_bert_${mode}_$TAG" -o run \
      --output-format csv -- python3 "$ROOT/bench/bert_bench.py" --steps 5 --warmup 3 > "$ROOT/gpurun_out/prof_bert_${mode}_$TAG.log" 2>&1 \
    || { echo "prof $mode failed"; tail -20 "$ROOT/gpurun_out/prof_bert_${mode}_$TAG.log"; exit 1; }
  echo "$mode ok"
done
