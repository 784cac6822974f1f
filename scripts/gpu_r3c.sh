#!/bin/bash
# BERT torch-op attribution (profiler with Python stacks, eager) and the 1-GPU async-PS rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-r3c}
timeout -k 10 300 python bench/bert_bench.py --steps 3 --warmup 3 --hip_graph 0 --trace_ops gpurun_out/bert_ops_$TAG \
    > gpurun_out/bert_ops_$TAG.json 2> gpurun_out/bert_ops_$TAG.err \
  || { echo "bert trace failed"; tail -20 gpurun_out/bert_ops_$TAG.err; exit 1; }
echo "bert trace ok"
if [ "${ASYNC:-1}" = 1 ]; then
timeout -k 10 500 python bench/async_ps_bench.py --share_gpu --num_ps 1 --num_workers 2 --depth 152 --batch 32 --image 160 \
    --steps 6 --warmup 2 --timeout_s 450 > gpurun_out/async_ps_$TAG.json 2> gpurun_out/async_ps_$TAG.err \
  || { echo "async failed"; tail -30 gpurun_out/async_ps_$TAG.err; exit 1; }
tail -1 gpurun_out/async_ps_$TAG.json | cut -c1-900
fi
timeout -k 10 200 python bench/conv_ws_probe.py --isolate --shapes 5,8 --tiles "4,8,1,3;2,8,1,3;4,8,2,3;2,8,2,3" \
    > gpurun_out/ws_iso_$TAG.txt 2>&1 || { echo "ws probe failed"; tail -20 gpurun_out/ws_iso_$TAG.txt; exit 1; }
cat gpurun_out/ws_iso_$TAG.txt | tail -30
cd /tmp
export TMPDIR=/tmp
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE"
P2="FETCH_SIZE TCC_HIT_sum GRBM_GUI_ACTIVE"
P3="TCC_MISS_sum WRITE_SIZE GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -d "$ROOT/gpurun_out/wspmc_${TAG}_p$i" -o run --output-format csv \
      -- python3 "$ROOT/bench/conv_ws_probe.py" --shapes 5,8 --tiles "4,8,1,3" > "$ROOT/gpurun_out/wspmc_${TAG}_p$i.log" 2>&1 \
      || { echo "ws pmc pass $i failed rc=$?"; tail -20 "$ROOT/gpurun_out/wspmc_${TAG}_p$i.log"; exit 1; }
  echo "ws pmc pass $i ok"
done
