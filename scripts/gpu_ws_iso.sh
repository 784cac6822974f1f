#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
TAG=${1:-iso}
TILES=${2:-4,4,1,4;2,8,1,4}
SHAPES=${3:-0,1,2,3,4,5,6,7,8,9,10}
timeout -k 10 300 python -u bench/conv_ws_probe.py --isolate --tiles "$TILES" --shapes "$SHAPES" \
    --out gpurun_out/probe_$TAG.json > gpurun_out/probe_$TAG.log 2>&1 || { tail -30 gpurun_out/probe_$TAG.log; exit 1; }
grep no_store gpurun_out/probe_$TAG.log | python -c "
import sys, json
for l in sys.stdin:
    r = json.loads(l); print(r['pass'], r['shape'], r['tile'], 'ws', r['ws_ms'], 'nostore', r['no_store_ms'], 'noload', r['no_load_ms'], 'compute', r['compute_only_ms'], 'store', r['store_only_ms'], 'load', r['load_only_ms'], 'cur', r['cur_ms'], 'floor', r['floor_ms'])
"
