#!/bin/bash
# GPU job: A/B of the BN-backward-statistics fusion (same box), plus the wgrad GEMM micro-bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-ab}
for v in 1 0 1 0; do
  MDTF_BN_BWD_STATS=$v timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_${TAG}_$v.log 2>&1 || exit 1
  echo "BN_BWD_STATS=$v $(tail -1 gpurun_out/bench_${TAG}_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 300 python bench/gemm_micro.py > gpurun_out/gemm_micro_$TAG.log 2>&1 || exit 1
cat gpurun_out/gemm_micro_$TAG.log
