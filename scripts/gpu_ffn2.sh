#!/bin/bash
# GPU job: BERT-base A/B of the fused FFN activation backward with the probed tile; rocprof of the fused step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2; do
  for f in 1 0; do
    MDTF_FFN_FUSE=$f timeout -k 10 300 python bench/bert_bench.py --steps 30 --warmup 5 > gpurun_out/bert_ffnb${f}_$i.json 2> gpurun_out/bert_ffnb${f}_$i.err \
        || { echo "bert failed"; tail -20 gpurun_out/bert_ffnb${f}_$i.err; exit 1; }
    echo "fuse=$f $i $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" gpurun_out/bert_ffnb${f}_$i.json)"
  done
done
R=$GRAFT_REPO_ROOT
cd /tmp && MDTF_FFN_FUSE=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_bert_ffn" -o run --output-format csv \
    -- python "$R/bench/bert_bench.py" --steps 5 --warmup 3 > "$R/gpurun_out/prof_bert_ffn.log" 2>&1 || { echo "prof failed"; exit 1; }
echo done
