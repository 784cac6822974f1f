#!/bin/bash
# GPU job: fused FFN activation-backward tests, tile probe, BERT-base A/B (fused vs separate act backward).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "dense or ffn or bert" --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_ffn.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_ffn.log; exit 1; }
tail -1 gpurun_out/pytest_ffn.log
timeout -k 10 300 python -u bench/dgrad_act_probe.py > gpurun_out/dgrad_act.jsonl 2> gpurun_out/dgrad_act.err \
    || { echo "probe failed"; tail -20 gpurun_out/dgrad_act.err; exit 1; }
cut -c1-400 gpurun_out/dgrad_act.jsonl
for i in 1 2; do
  for f in 1 0; do
    MDTF_FFN_FUSE=$f timeout -k 10 300 python bench/bert_bench.py --steps 30 --warmup 5 > gpurun_out/bert_ffn${f}_$i.json 2> gpurun_out/bert_ffn${f}_$i.err \
        || { echo "bert failed"; tail -20 gpurun_out/bert_ffn${f}_$i.err; exit 1; }
    echo "fuse=$f $i $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('loss_last'))" gpurun_out/bert_ffn${f}_$i.json)"
  done
done
