#!/bin/bash
# GPU job: ResNet-50 and BERT-base benches + rocprofv3 kernel traces of both (graph-captured steps).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-fin}
timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
timeout -k 10 200 python bench/bert_bench.py --steps 30 --warmup 5 > gpurun_out/bert_$TAG.json 2> gpurun_out/bert_$TAG.err || { tail -20 gpurun_out/bert_$TAG.err; exit 1; }
cat gpurun_out/bert_$TAG.json
timeout -k 10 200 python bench/bert_bench.py --steps 30 --warmup 5 --stock > gpurun_out/bert_stock_$TAG.json 2> gpurun_out/bert_stock_$TAG.err || { tail -20 gpurun_out/bert_stock_$TAG.err; exit 1; }
cat gpurun_out/bert_stock_$TAG.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_rn_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --steps 5 --warmup 3 > "$ROOT/gpurun_out/prof_rn_$TAG.log" 2>&1 || { echo "resnet prof failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_bert_$TAG" -o run --output-format csv -- python3 "$ROOT/bench/bert_bench.py" --steps 5 --warmup 3 > "$ROOT/gpurun_out/prof_bert_$TAG.log" 2>&1 || { echo "bert prof failed"; exit 1; }
echo "profiles done"
