#!/bin/bash
# A/B of an environment setting on the BERT-base bench: VAR=A vs VAR=B, alternating, 2 runs each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=$1; VAR=$2; A=$3; B=$4; shift 4
for i in 1 2; do
  for v in "$A" "$B"; do
    env "$VAR=$v" timeout -k 10 300 python bench/bert_bench.py --steps 30 --warmup 5 "$@" > gpurun_out/bab_${TAG}_$v$i.json \
        2> gpurun_out/bab_${TAG}_$v$i.err || { echo "bert $v failed"; tail -20 gpurun_out/bab_${TAG}_$v$i.err; exit 1; }
    echo "$VAR=$v run $i: $(python -c "import json; d=json.loads(open('gpurun_out/bab_${TAG}_$v$i.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
  done
done
