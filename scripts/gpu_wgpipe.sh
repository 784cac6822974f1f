#!/bin/bash
# Pipelined conv_wgrad_v2 main loop: numerics tests, then an A/B timing sweep (MDTF_WGRAD_PIPE=1 vs 0).
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
cd "$ROOT"
TAG=${1:-p1}
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "wgrad or conv_hip or engine_step" --timeout 120 --timeout-method thread > "$OUT/wgpipe_${TAG}_tests.log" 2>&1 || { echo "tests rc=$?"; tail -30 "$OUT/wgpipe_${TAG}_tests.log"; exit 1; }
tail -3 "$OUT/wgpipe_${TAG}_tests.log"
MDTF_WGRAD_PIPE=1 timeout -k 10 300 python3 bench/wgrad_probe.py --quick > "$OUT/wgpipe_${TAG}_on.md" 2>&1 || { echo "probe on rc=$?"; tail -20 "$OUT/wgpipe_${TAG}_on.md"; exit 1; }
MDTF_WGRAD_PIPE=0 timeout -k 10 300 python3 bench/wgrad_probe.py --quick > "$OUT/wgpipe_${TAG}_off.md" 2>&1 || { echo "probe off rc=$?"; exit 1; }
grep best "$OUT/wgpipe_${TAG}_on.md" "$OUT/wgpipe_${TAG}_off.md"
