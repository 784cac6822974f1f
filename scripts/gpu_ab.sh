#!/bin/bash
# A/B: ResNet-50 bench with conv table A vs B (alternating, 2 runs each), one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-ab}; A=${2:-bench/conv_table_prev.json}; B=${3:-mdtf/ops/conv_table.json}
for i in 1 2; do
  for T in A B; do
    F=$A; [ $T = B ] && F=$B
    MDTF_CONV_TABLE=$F timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/ab_${TAG}_$T$i.json \
        2> gpurun_out/ab_${TAG}_$T$i.err || { echo "bench $T failed"; tail -20 gpurun_out/ab_${TAG}_$T$i.err; exit 1; }
    echo "$T$i $(python -c "import json,sys; d=json.load(open('gpurun_out/ab_${TAG}_$T$i.json')); print(d['value'], d['ms_per_step'])")"
  done
done
