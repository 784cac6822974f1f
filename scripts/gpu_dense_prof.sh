#!/bin/bash
# GPU job: BN tests + ResNet-50 bench (dual-BN backward change), rocprof of BERT-base with the hand-written
# vs library dense forward (per-kernel times inside the step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-dp}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v -m gpu -k "batch_norm or resnet" --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_$TAG.log
# test failures (rc 1) are read afterwards; anything else (crash, time limit) ends the job
[ $rc -le 1 ] || { echo "pytest rc=$rc"; exit 1; }
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --bert 0 > gpurun_out/bench_$TAG$i.json 2> gpurun_out/bench_$TAG$i.err \
    || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG$i.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('resnet', d['value'], d['ms_per_step'])" gpurun_out/bench_$TAG$i.json
done
for mode in mdtf hipblaslt; do
  cd /tmp && MDTF_DENSE_FWD=$mode timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_bert_${TAG}_$mode" -o run \
      --output-format csv -- python "$GRAFT_REPO_ROOT/bench/bert_bench.py" --steps 5 --warmup 3 > "$GRAFT_REPO_ROOT/gpurun_out/prof_bert_${TAG}_$mode.log" 2>&1 \
      || { echo "prof $mode failed"; tail -20 "$GRAFT_REPO_ROOT/gpurun_out/prof_bert_${TAG}_$mode.log"; exit 1; }
  cd "$GRAFT_REPO_ROOT"
done
echo done
