#!/bin/bash
# Round-3 GPU job: GEMM-core numerics, the GPU tests of the new dense core / attention / hipGraph+RCCL capture,
# BERT-base A/B (ping-pong core vs the r2 mix), the headline bench, and the 1-GPU async-PS rehearsal.
# Stops at the first failing GPU step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-r3}
STEPS=${STEPS:-all}
step() { echo "== $1 $(date +%T)"; }
step check
timeout -k 10 240 python -u bench/gemm_pp_probe.py --check > gpurun_out/gemm_check_$TAG.jsonl 2> gpurun_out/gemm_check_$TAG.err \
  || { echo "check failed"; grep -v '"ok": true' gpurun_out/gemm_check_$TAG.jsonl | cut -c1-250 | head; tail -5 gpurun_out/gemm_check_$TAG.err; exit 1; }
grep -c '"ok": true' gpurun_out/gemm_check_$TAG.jsonl
step tests
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "dense or ffn or bert or gemm or attention or apply_multi or backup" \
    --timeout 150 --timeout-method thread > gpurun_out/pytest_dense_$TAG.log 2>&1 \
  || { echo "pytest failed"; tail -40 gpurun_out/pytest_dense_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_dense_$TAG.log
# the RCCL-in-hipGraph tests with output uncaptured (-s): a native abort prints its cause into the log
timeout -k 10 300 python -u -m pytest tests/test_hip_graph.py -x -v -s -m gpu --timeout 150 --timeout-method thread \
    > gpurun_out/pytest_graph_$TAG.log 2>&1 || { echo "graph tests failed rc=$?"; tail -40 gpurun_out/pytest_graph_$TAG.log; exit 1; }
grep -E "passed|failed" gpurun_out/pytest_graph_$TAG.log | tail -1
[ "$STEPS" = "tests" ] && exit 0
step bert
for mode in pp legacy; do
  MDTF_DENSE=$mode timeout -k 10 300 python bench/bert_bench.py --steps 20 --warmup 5 > gpurun_out/bert_${mode}_$TAG.json 2> gpurun_out/bert_${mode}_$TAG.err \
      || { echo "bert $mode failed"; tail -20 gpurun_out/bert_${mode}_$TAG.err; exit 1; }
  echo "$mode $(tail -1 gpurun_out/bert_${mode}_$TAG.json | cut -c1-160)"
done
MDTF_ATTN_FLASH=1 timeout -k 10 300 python bench/bert_bench.py --steps 20 --warmup 5 > gpurun_out/bert_flash_$TAG.json 2> gpurun_out/bert_flash_$TAG.err \
    || { echo "bert flash failed"; tail -20 gpurun_out/bert_flash_$TAG.err; exit 1; }
echo "pp+flash128 $(tail -1 gpurun_out/bert_flash_$TAG.json | cut -c1-160)"
step bench
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --bert 0 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
  || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.err; exit 1; }
tail -1 gpurun_out/bench_$TAG.json | cut -c1-300
[ "$STEPS" = "noasync" ] && exit 0
step async
timeout -k 10 500 python bench/async_ps_bench.py --share_gpu --num_ps 1 --num_workers 2 --depth 152 --batch 32 --image 160 \
    --steps 6 --warmup 2 --timeout_s 450 > gpurun_out/async_ps_$TAG.json 2> gpurun_out/async_ps_$TAG.err \
  || { echo "async failed"; tail -30 gpurun_out/async_ps_$TAG.err; exit 1; }
tail -1 gpurun_out/async_ps_$TAG.json | cut -c1-600
