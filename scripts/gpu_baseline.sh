#!/bin/bash
# GPU job: comparator + framework (torch kernels) baseline + rocprof kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 240 python -c "import torch;print(torch.cuda.get_device_name(0), torch.version.hip)" > gpurun_out/dev.txt 2>&1 &&
timeout -k 10 300 python bench/stock_pytorch.py --steps 20 --warmup 5 > gpurun_out/stock.json 2> gpurun_out/stock.err &&
timeout -k 10 300 python bench.py --kernels torch --steps 20 --warmup 5 > gpurun_out/bench_torch.json 2> gpurun_out/bench_torch.err &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_torch -o run --output-format csv -- python bench.py --kernels torch --steps 5 --warmup 3 > gpurun_out/prof_torch.log 2>&1
echo "exit $?"
