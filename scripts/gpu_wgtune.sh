#!/bin/bash
# Re-tune the weight-gradient entries of the conv table with the current kernels, then A/B the bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
TAG=${1:-wgt}
cp mdtf/ops/conv_table.json gpurun_out/conv_table_$TAG.json
timeout -k 10 700 python -u bench/conv_autotune.py --passes wgrad --merge --out gpurun_out/conv_table_$TAG.json \
    --report gpurun_out/conv_autotune_$TAG.md > gpurun_out/tune_$TAG.log 2>&1 || { echo "autotune failed"; tail -30 gpurun_out/tune_$TAG.log; exit 1; }
tail -2 gpurun_out/tune_$TAG.log
for i in 1 2; do
  for t in mdtf/ops/conv_table.json gpurun_out/conv_table_$TAG.json; do
    MDTF_CONV_TABLE=$t timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/wgt_${TAG}_$i.json 2> gpurun_out/wgt_${TAG}_$i.err || { echo "bench failed"; tail -20 gpurun_out/wgt_${TAG}_$i.err; exit 1; }
    echo "$t run $i: $(python -c "import json; d=json.load(open('gpurun_out/wgt_${TAG}_$i.json')); print(d['value'], d['ms_per_step'])")"
  done
done
