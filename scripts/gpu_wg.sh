#!/bin/bash
# Weight-gradient kernel: numerics, then the graph-timed sweep over the BERT shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-wg}
timeout -k 10 180 python -u bench/gemm_wg_probe.py --check > gpurun_out/wg_check_$TAG.jsonl 2> gpurun_out/wg_check_$TAG.err \
  || { echo "check failed"; grep -v '"ok": true' gpurun_out/wg_check_$TAG.jsonl | head -20; tail -5 gpurun_out/wg_check_$TAG.err; exit 1; }
echo "check ok: $(grep -c '"ok": true' gpurun_out/wg_check_$TAG.jsonl)"
timeout -k 10 300 python -u bench/gemm_wg_probe.py ${SHAPES:+--shapes $SHAPES} > gpurun_out/wg_probe_$TAG.jsonl 2> gpurun_out/wg_probe_$TAG.err \
  || { echo "probe failed"; tail -5 gpurun_out/wg_probe_$TAG.err; exit 1; }
python - <<'PY' gpurun_out/wg_probe_$TAG.jsonl
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["shape"], "best", d["best"], d["best_tf"], "pick", d["pick"], d["pick_tf"], "lib", d["lib_tf"], "r2", d["r2_tf"])
PY
