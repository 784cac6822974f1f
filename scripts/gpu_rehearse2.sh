#!/bin/bash
# GPU job: 2-rank rehearsal of the headline bench on ONE GPU (gloo backend, both ranks share the device): the
# self-launch, per-rank device, bucketed gradient all-reduce on device tensors, eager step (gloo is not
# capturable), max-over-ranks timing and the JSON line.  Not a scaling measurement.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
MDTF_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --bert 0 \
    > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err || { echo "rehearsal failed rc=$?"; tail -30 gpurun_out/rehearse2.err; exit 1; }
tail -1 gpurun_out/rehearse2.json | cut -c1-400
MDTF_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --bert 0 --mode sharded --comm_dtype bf16 \
    > gpurun_out/rehearse2s.json 2> gpurun_out/rehearse2s.err || { echo "sharded rehearsal failed rc=$?"; tail -30 gpurun_out/rehearse2s.err; exit 1; }
tail -1 gpurun_out/rehearse2s.json | cut -c1-400
