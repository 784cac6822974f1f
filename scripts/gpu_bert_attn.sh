#!/bin/bash
# GPU job: BERT-base benches -- seq 128 with the whole-sequence attention kernels and with the tiled ones,
# seq 512 (phase 2) on the tiled kernels, and the stock comparator at seq 512.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-ba}
run() { timeout -k 10 240 python bench/bert_bench.py --steps 20 --warmup 5 "$@" 2>/dev/null | tail -1; }
echo "seq128 default: $(run)"
echo "seq128 flash:   $(MDTF_ATTN_FLASH=1 run)"
echo "seq512 b16:     $(run --seq 512 --batch 16)"
echo "seq512 stock:   $(run --seq 512 --batch 16 --stock)"
