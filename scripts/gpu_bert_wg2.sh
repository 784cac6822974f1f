#!/bin/bash
# GPU job: dense wgrad tests + BERT-base with the re-tuned dense weight-gradient tiles; then the graph-timed conv
# re-tune and its ResNet-50 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "wgrad or dense or bert" --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_wg2.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_wg2.log; exit 1; }
tail -1 gpurun_out/pytest_wg2.log
for i in 1 2; do
  timeout -k 10 300 python bench/bert_bench.py --steps 30 --warmup 5 > gpurun_out/bert_wg2_$i.json 2> gpurun_out/bert_wg2_$i.err \
      || { echo "bert failed"; tail -20 gpurun_out/bert_wg2_$i.err; exit 1; }
  echo "bert $i $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])" gpurun_out/bert_wg2_$i.json)"
done
bash scripts/gpu_tune_graph.sh
