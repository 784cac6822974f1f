#!/bin/bash
# GPU job: 1-GPU ResNet-50 bench (2 runs) + one rocprofv3 kernel-trace run of the bench.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-bp}
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_${TAG}_$i.json 2> gpurun_out/bench_${TAG}_$i.err \
      || { echo "bench failed"; tail -20 gpurun_out/bench_${TAG}_$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_${TAG}_$i.json')); print(d['value'], d['ms_per_step'])"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_$TAG" -o run --output-format csv \
    -- python3 "$ROOT/bench.py" --steps 5 --warmup 3 > "$ROOT/gpurun_out/prof_$TAG.log" 2>&1
echo "prof exit $?"
