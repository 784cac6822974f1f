#!/bin/bash
# GPU job: full GPU suite, ResNet-50 bench x2, graph-timed dense probe, kernel-only time vs stock.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-r2g}
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_$TAG.log
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --bert 0 > gpurun_out/bench_$TAG$i.json 2> gpurun_out/bench_$TAG$i.err \
    || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG$i.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('resnet', d['value'], d['ms_per_step'], d['loss_last'])" gpurun_out/bench_$TAG$i.json
done
timeout -k 10 300 python -u bench/dense_fwd_probe.py > gpurun_out/probe_$TAG.jsonl 2> gpurun_out/probe_$TAG.err \
    || { echo "probe failed"; tail -20 gpurun_out/probe_$TAG.err; exit 1; }
cut -c1-220 gpurun_out/probe_$TAG.jsonl
bash scripts/gpu_kernel_vs_stock.sh
