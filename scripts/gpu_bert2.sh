#!/bin/bash
# GPU job: transformer/GEMM tests, BERT bench (mdtf) + rocprof of it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-bert2}
timeout -k 10 600 python -m pytest tests -q -m gpu -k "bert or colsum or layernorm or bias_act or softmax or embedding or engine or attention or wgrad" > gpurun_out/pytest_gpu_$TAG.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_gpu_$TAG.log
tail -3 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python bench/bert_bench.py --steps 20 --warmup 5 > gpurun_out/bert_$TAG.json 2> gpurun_out/bert_$TAG.err &&
cat gpurun_out/bert_$TAG.json &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert_$TAG -o run --output-format csv -- python bench/bert_bench.py --steps 5 --warmup 3 > gpurun_out/prof_bert_$TAG.log 2>&1
echo "exit $?"
