#!/bin/bash
# GPU job: conv tests (incl. strided v2 dgrad), stride-2 dgrad autotune merged into the table, bench, PMC
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-s3}
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py tests/test_kernels_property.py -q -m gpu -k "conv" \
  > gpurun_out/pytest_conv_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_conv_$TAG.log; exit 1; }
tail -2 gpurun_out/pytest_conv_$TAG.log
cp mdtf/ops/conv_table.json gpurun_out/conv_table_$TAG.json
timeout -k 10 600 python bench/conv_autotune.py --passes dgrad --strides 2 --merge --reps 8 \
  --out gpurun_out/conv_table_$TAG.json --report gpurun_out/conv_autotune_$TAG.md > gpurun_out/autotune_$TAG.log 2>&1 \
  || { tail -20 gpurun_out/autotune_$TAG.log; exit 1; }
tail -2 gpurun_out/autotune_$TAG.log
cp gpurun_out/conv_table_$TAG.json mdtf/ops/conv_table.json
timeout -k 10 400 python bench.py --steps 30 --warmup 10 > gpurun_out/bench_$TAG.log 2>&1 || { tail -20 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT \
  --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG" -o run -- python3 "$GRAFT_REPO_ROOT/scripts/conv_pmc.py" \
  > "$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG.log"; exit 1; }
echo done
