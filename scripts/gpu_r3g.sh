#!/bin/bash
# Round-3 GEMM diagnosis: graph-timed GEMM-core vs hipBLASLt on the BERT / square shapes, one counter pass over
# the core variants, then kernel stats + one SQ counter pass over the ResNet-50 and BERT-base steps.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"
mkdir -p gpurun_out
TAG=${1:-g1}
timeout -k 10 300 python -u bench/gemm_pp_probe.py > gpurun_out/gemm_probe_$TAG.jsonl 2> gpurun_out/gemm_probe_$TAG.err \
  || { echo "probe failed"; tail -5 gpurun_out/gemm_probe_$TAG.err; exit 1; }
echo "probe ok"
bash scripts/gpu_gemm_pmc.sh gpmc_$TAG || exit 1
[ -n "$PROF" ] && { bash scripts/gpu_prof_r3.sh $TAG || exit 1; }
echo done
