#!/bin/bash
# One rocprofv3 counter pass over the GEMM-core variants (bench/gemm_pp_pmc.py).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$ROOT/gpurun_out"
export TMPDIR=/tmp
TAG=${1:-gpmc}
cd /tmp
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace -d "$ROOT/gpurun_out/${TAG}" -o run --output-format csv \
    -- python3 "$ROOT/bench/gemm_pp_pmc.py" > "$ROOT/gpurun_out/${TAG}.log" 2>&1 \
    || { echo "pmc pass failed rc=$?"; tail -20 "$ROOT/gpurun_out/${TAG}.log"; exit 1; }
echo "pmc ok"
