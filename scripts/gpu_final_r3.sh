#!/bin/bash
# Round-3 evidence on the current build: kernel stats of the captured BERT-base / ResNet-50 steps, then SQ, fetch
# and write/L2 counter passes over each (eager; one counter group per run, each under its own kill timer).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$ROOT/gpurun_out"
export TMPDIR=/tmp
TAG=${1:-f3}
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_bert_$TAG" -o run --output-format csv \
    -- python3 "$ROOT/bench/bert_bench.py" --steps 5 --warmup 3 > "$ROOT/gpurun_out/prof_bert_$TAG.log" 2>&1 \
  || { echo "bert prof failed"; tail -20 "$ROOT/gpurun_out/prof_bert_$TAG.log"; exit 1; }
echo "bert stats ok"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_resnet_$TAG" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 5 --warmup 3 --bert 0 > "$ROOT/gpurun_out/prof_resnet_$TAG.log" 2>&1 \
  || { echo "resnet prof failed"; tail -20 "$ROOT/gpurun_out/prof_resnet_$TAG.log"; exit 1; }
echo "resnet stats ok"
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
P2="FETCH_SIZE GRBM_GUI_ACTIVE"
P3="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace -d "$ROOT/gpurun_out/pmcb_${TAG}_p$i" -o run --output-format csv \
      -- python3 "$ROOT/bench/bert_bench.py" --steps 2 --warmup 1 --hip_graph 0 > "$ROOT/gpurun_out/pmcb_${TAG}_p$i.log" 2>&1 \
    || { echo "bert pmc $i failed"; tail -20 "$ROOT/gpurun_out/pmcb_${TAG}_p$i.log"; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace -d "$ROOT/gpurun_out/pmcr_${TAG}_p$i" -o run --output-format csv \
      -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --hip_graph 0 --bert 0 > "$ROOT/gpurun_out/pmcr_${TAG}_p$i.log" 2>&1 \
    || { echo "resnet pmc $i failed"; tail -20 "$ROOT/gpurun_out/pmcr_${TAG}_p$i.log"; exit 1; }
  echo "pmc pass $i ok"
done
