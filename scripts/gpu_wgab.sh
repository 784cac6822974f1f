#!/bin/bash
# GPU job: BN backward-statistics trace; BERT-base A/B of the dense weight gradient (hand-written vs hipBLASLt).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/bn_trace.py > gpurun_out/bn_trace.log 2>&1 || { echo "bn_trace failed"; tail -20 gpurun_out/bn_trace.log; exit 1; }
tail -12 gpurun_out/bn_trace.log
for i in 1 2; do
  for mode in mdtf hipblaslt; do
    MDTF_DENSE_WGRAD=$mode timeout -k 10 300 python bench/bert_bench.py --steps 30 --warmup 5 > gpurun_out/bertwg_${mode}_$i.json 2> gpurun_out/bertwg_${mode}_$i.err \
        || { echo "bert failed"; tail -20 gpurun_out/bertwg_${mode}_$i.err; exit 1; }
    echo "wgrad=$mode $i $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" gpurun_out/bertwg_${mode}_$i.json)"
  done
done
