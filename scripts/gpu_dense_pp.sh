#!/bin/bash
# GPU job: GEMM-core numerics, the dense/BERT GPU tests on the new core, BERT-base bench A/B (pp vs legacy).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-d}
timeout -k 10 240 python -u bench/gemm_pp_probe.py --check > gpurun_out/gemm_check_$TAG.jsonl 2> gpurun_out/gemm_check_$TAG.err
rc=$?
grep -c '"ok": true' gpurun_out/gemm_check_$TAG.jsonl; grep -v '"ok": true' gpurun_out/gemm_check_$TAG.jsonl | cut -c1-250 | head -5
[ $rc -eq 0 ] || { echo "check rc=$rc"; tail -20 gpurun_out/gemm_check_$TAG.err; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "dense or ffn or bert or gemm" --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_dense_$TAG.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_dense_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_dense_$TAG.log
for mode in pp legacy; do
  MDTF_DENSE=$mode timeout -k 10 300 python bench/bert_bench.py --steps 20 --warmup 5 > gpurun_out/bert_${mode}_$TAG.json 2> gpurun_out/bert_${mode}_$TAG.err \
      || { echo "bert $mode failed"; tail -20 gpurun_out/bert_${mode}_$TAG.err; exit 1; }
  echo "$mode $(tail -1 gpurun_out/bert_${mode}_$TAG.json | cut -c1-200)"
done
