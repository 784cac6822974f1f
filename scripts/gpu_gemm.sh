#!/bin/bash
# GPU job: numerics of the ping-pong GEMM core, then its graph-timed speed vs hipBLASLt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-a}
timeout -k 10 240 python -u bench/gemm_pp_probe.py --check > gpurun_out/gemm_check_$TAG.jsonl 2> gpurun_out/gemm_check_$TAG.err
rc=$?
cut -c1-220 gpurun_out/gemm_check_$TAG.jsonl | tail -25
[ $rc -eq 0 ] || { echo "check rc=$rc"; tail -20 gpurun_out/gemm_check_$TAG.err; exit 1; }
timeout -k 10 400 python -u bench/gemm_pp_probe.py ${SHAPES:+--shapes $SHAPES} > gpurun_out/gemm_bench_$TAG.jsonl 2> gpurun_out/gemm_bench_$TAG.err \
  || { echo "bench failed"; tail -20 gpurun_out/gemm_bench_$TAG.err; exit 1; }
cat gpurun_out/gemm_bench_$TAG.jsonl
