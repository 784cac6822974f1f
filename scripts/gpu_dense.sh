#!/bin/bash
# GPU job: dense forward kernel tests, shape probe vs hipBLASLt, BERT-base A/B (hand-written vs library forward).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-dense}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -m gpu -k "dense" --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_$TAG.log
timeout -k 10 300 python -u bench/dense_fwd_probe.py > gpurun_out/probe_$TAG.jsonl 2> gpurun_out/probe_$TAG.err \
    || { echo "probe failed"; tail -20 gpurun_out/probe_$TAG.err; exit 1; }
cat gpurun_out/probe_$TAG.jsonl
for i in 1 2; do
  for mode in mdtf hipblaslt; do
    MDTF_DENSE_FWD=$mode timeout -k 10 300 python bench/bert_bench.py --steps 30 --warmup 5 > gpurun_out/bert_${TAG}_${mode}_$i.json 2> gpurun_out/bert_${TAG}_${mode}_$i.err \
        || { echo "bert failed"; tail -20 gpurun_out/bert_${TAG}_${mode}_$i.err; exit 1; }
    echo "$mode $i $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" gpurun_out/bert_${TAG}_${mode}_$i.json)"
  done
done
