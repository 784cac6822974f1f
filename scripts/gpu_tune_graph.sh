#!/bin/bash
# GPU job: re-tune the conv table with graph-timed candidates, then A/B the ResNet-50 step (new vs shipped table).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 900 python -u bench/conv_autotune.py --graph --reps 10 --out gpurun_out/conv_table_graph.json \
    --report gpurun_out/conv_autotune_graph.md > gpurun_out/tune_graph.log 2>&1 \
    || { echo "autotune failed"; tail -30 gpurun_out/tune_graph.log; exit 1; }
tail -2 gpurun_out/tune_graph.log
for i in 1 2 3; do
  for t in shipped graph; do
    if [ $t = graph ]; then export MDTF_CONV_TABLE=$PWD/gpurun_out/conv_table_graph.json; else unset MDTF_CONV_TABLE; fi
    timeout -k 10 300 python bench.py --steps 30 --warmup 5 --bert 0 > gpurun_out/tab_${t}_$i.json 2> gpurun_out/tab_${t}_$i.err \
        || { echo "bench failed"; tail -20 gpurun_out/tab_${t}_$i.err; exit 1; }
    echo "$t $i $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" gpurun_out/tab_${t}_$i.json)"
  done
done
