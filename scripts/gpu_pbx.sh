#!/bin/bash
# GPU job: dgrad BN-statistics prefetch (MDTF_DGRAD_PBX) tests + ResNet-50 A/B, then the full round check.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "conv or batch_norm or resnet or bn or stats" --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_pbx.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_pbx.log; exit 1; }
tail -1 gpurun_out/pytest_pbx.log
for i in 1 2 3; do
  for f in 1 0; do
    MDTF_DGRAD_PBX=$f timeout -k 10 300 python bench.py --steps 30 --warmup 5 --bert 0 > gpurun_out/pbx${f}_$i.json 2> gpurun_out/pbx${f}_$i.err \
        || { echo "bench failed"; tail -20 gpurun_out/pbx${f}_$i.err; exit 1; }
    echo "pbx=$f $i $(python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['loss_last'])" gpurun_out/pbx${f}_$i.json)"
  done
done
PROF=1 bash scripts/gpu_round.sh r2j
