#!/bin/bash
# GPU job: MODE 4 (prefetched activation-backward epilogue) tests + probe + BERT A/B, then the 2-rank one-GPU
# gloo rehearsal of bench.py.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "dense or ffn or bert or resnet" --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_m4.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_m4.log; exit 1; }
tail -1 gpurun_out/pytest_m4.log
timeout -k 10 300 python -u bench/dgrad_act_probe.py > gpurun_out/dgrad_act_m4.jsonl 2> gpurun_out/dgrad_act_m4.err \
    || { echo "probe failed"; tail -20 gpurun_out/dgrad_act_m4.err; exit 1; }
cut -c1-300 gpurun_out/dgrad_act_m4.jsonl
for i in 1 2; do
  for f in 1 0; do
    MDTF_FFN_FUSE=$f timeout -k 10 300 python bench/bert_bench.py --steps 30 --warmup 5 > gpurun_out/bert_m4${f}_$i.json 2> gpurun_out/bert_m4${f}_$i.err \
        || { echo "bert failed"; tail -20 gpurun_out/bert_m4${f}_$i.err; exit 1; }
    echo "fuse=$f $i $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" gpurun_out/bert_m4${f}_$i.json)"
  done
done
bash scripts/gpu_rehearse2.sh
