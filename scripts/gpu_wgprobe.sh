#!/bin/bash
# conv_wgrad_v2 probe: timing sweep, then counter passes over two configs.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$ROOT"
timeout -k 10 400 python3 bench/wgrad_probe.py > "$OUT/wgprobe.md" 2> "$OUT/wgprobe.err" || { echo "sweep rc=$?"; tail -20 "$OUT/wgprobe.err"; exit 1; }
cd /tmp
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
P2="FETCH_SIZE GRBM_GUI_ACTIVE"
P3="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
i=0
for CFG in "8192 4096 4096 256 256 2 3 1 0" "8192 768 3072 256 256 2 3 8 1" "8192 768 3072 64 128 2 2 4 1"; do
  i=$((i+1)); j=0
  for P in "$P1" "$P2" "$P3"; do
    j=$((j+1))
    timeout -s KILL 60 rocprofv3 --pmc $P --kernel-trace -d "$OUT/wgpmc_c${i}_p$j" -o run --output-format csv \
      -- python3 "$ROOT/bench/wgrad_probe.py" --one $CFG > "$OUT/wgpmc_c${i}_p$j.log" 2>&1 \
      || { echo "cfg $i pass $j failed"; tail -20 "$OUT/wgpmc_c${i}_p$j.log"; exit 1; }
  done
  echo "cfg $i ok"
done
