#!/bin/bash
# Counter passes over the weight-gradient kernel configs (bench/gemm_wg_pmc.py), one pass per counter group.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p "$ROOT/gpurun_out"
export TMPDIR=/tmp
TAG=${1:-wgpmc}
cd /tmp
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE"
P2="FETCH_SIZE GRBM_GUI_ACTIVE"
P3="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -d "$ROOT/gpurun_out/${TAG}_p$i" -o run --output-format csv \
      -- python3 "$ROOT/bench/gemm_wg_pmc.py" > "$ROOT/gpurun_out/${TAG}_p$i.log" 2>&1 \
      || { echo "pass $i failed rc=$?"; tail -20 "$ROOT/gpurun_out/${TAG}_p$i.log"; exit 1; }
  echo "pass $i ok"
done
