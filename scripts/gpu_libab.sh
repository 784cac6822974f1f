#!/bin/bash
# A/B of two kernel-library builds on one box: the in-tree build vs mdtf/csrc/build/libmdtf_kernels_ab.so.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
TAG=${1:-lab}
for i in 1 2; do
  for v in new old; do
    if [ "$v" = old ]; then L="$ROOT/mdtf/csrc/build/libmdtf_kernels_ab.so"; else L=""; fi
    MDTF_KERNELS_LIB="$L" timeout -k 10 200 python bench.py --steps 30 --warmup 5 --bert 0 > gpurun_out/lab_${TAG}_rn_$v$i.json 2> gpurun_out/lab_${TAG}_rn_$v$i.err || { echo "resnet $v failed"; tail -20 gpurun_out/lab_${TAG}_rn_$v$i.err; exit 1; }
    MDTF_KERNELS_LIB="$L" timeout -k 10 200 python bench/bert_bench.py --steps 30 --warmup 5 > gpurun_out/lab_${TAG}_bert_$v$i.json 2> gpurun_out/lab_${TAG}_bert_$v$i.err || { echo "bert $v failed"; tail -20 gpurun_out/lab_${TAG}_bert_$v$i.err; exit 1; }
    echo "$v run $i: resnet $(python -c "import json; print(json.load(open('gpurun_out/lab_${TAG}_rn_$v$i.json'))['value'])") bert $(python -c "import json; print(json.load(open('gpurun_out/lab_${TAG}_bert_$v$i.json'))['value'])")"
  done
done
