#!/bin/bash
# GPU job: the ResNet-50 gradient test with the shortcut BN backward reading dy+mask (default) vs the written dz
# copy (MDTF_DUAL_DZ=1), twice each; then the dense-prof job.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2; do
  for dz in 0 1; do
    MDTF_DUAL_DZ=$dz timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "resnet50_step_loss" --timeout 120 --timeout-method thread \
      > gpurun_out/ab_dual_${dz}_$i.log 2>&1
    echo "dz=$dz run $i rc=$? $(grep -E 'AssertionError:|passed|failed' gpurun_out/ab_dual_${dz}_$i.log | head -3 | tr '\n' ' ')"
  done
done
