#!/bin/bash
# hipBLASLt/rocBLAS solution tuning of BERT's GEMMs with PyTorch TunableOp, then an A/B of the tuned table.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$ROOT"; mkdir -p gpurun_out
TAG=${1:-tu}
F="$ROOT/gpurun_out/tunableop_${TAG}%d.csv"
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME="$F" \
  timeout -k 10 700 python bench/bert_bench.py --steps 3 --warmup 3 > gpurun_out/tu_${TAG}_tune.json 2> gpurun_out/tu_${TAG}_tune.err || { echo "tuning failed"; tail -20 gpurun_out/tu_${TAG}_tune.err; exit 1; }
ls -la gpurun_out/tunableop_${TAG}*.csv
for i in 1 2; do
  for v in tuned plain; do
    if [ "$v" = tuned ]; then E="PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$F"; else E="PYTORCH_TUNABLEOP_ENABLED=0"; fi
    env $E timeout -k 10 200 python bench/bert_bench.py --steps 30 --warmup 5 > gpurun_out/tu_${TAG}_$v$i.json 2> gpurun_out/tu_${TAG}_$v$i.err || { echo "bert $v failed"; tail -20 gpurun_out/tu_${TAG}_$v$i.err; exit 1; }
    echo "$v run $i: $(python -c "import json; print(json.load(open('gpurun_out/tu_${TAG}_$v$i.json'))['value'])")"
  done
done
