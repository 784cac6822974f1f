#!/bin/bash
# A/B of an environment setting on both benches (ResNet-50 bench.py, BERT-base bert_bench.py), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=$1; VAR=$2; A=$3; B=$4
for i in 1 2; do
  for v in "$A" "$B"; do
    env "$VAR=$v" timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/bab_${TAG}_rn_$v$i.json \
        2> gpurun_out/bab_${TAG}_rn_$v$i.err || { echo "resnet $v failed"; tail -20 gpurun_out/bab_${TAG}_rn_$v$i.err; exit 1; }
    env "$VAR=$v" timeout -k 10 200 python bench/bert_bench.py --steps 30 --warmup 5 > gpurun_out/bab_${TAG}_bert_$v$i.json \
        2> gpurun_out/bab_${TAG}_bert_$v$i.err || { echo "bert $v failed"; tail -20 gpurun_out/bab_${TAG}_bert_$v$i.err; exit 1; }
    echo "$VAR=$v run $i: resnet $(python -c "import json; print(json.load(open('gpurun_out/bab_${TAG}_rn_$v$i.json'))['value'])") bert $(python -c "import json; print(json.load(open('gpurun_out/bab_${TAG}_bert_$v$i.json'))['value'])")"
  done
done
