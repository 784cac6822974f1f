#!/bin/bash
# One entry point for the GPU-box runs (gpurun -- bash scripts/gpu.sh <what> [tag] [extra args]).
#   tests   : pytest -m gpu (one process, per-test timeout)
#   bench   : bench.py (ResNet-50 + BERT-base line), three times
#   prof    : rocprofv3 --kernel-trace --stats of the captured ResNet-50 and BERT-base steps
#   profr   : the same, ResNet-50 only
#   pmc     : SQ / FETCH / WRITE+L2 counter passes over both steps (captured steps; PMC_GRAPH=0: eager), each its
#             own run; summarise one step with scripts/pmc_summary.py <dir prefix> 40 --last-step
#   envab   : alternating A/B of bench.py under two env settings: gpu.sh envab TAG "A=1" "A=0" [steps]
#   py      : run a python script under a time limit: gpu.sh py TAG path/to/script.py [args]
#   bertab  : alternating A/B of bench/bert_bench.py under two env settings: gpu.sh bertab TAG "A=1" "A=0" [steps]
#   rehearse2: 2-rank gloo rehearsal of bench.py on the one GPU (allreduce and sharded/bf16 modes; not a scaling run)
#   final   : tests + bench (30 steps, three runs) + prof of the tree, stopping at the first failure (the sequence
#             every round-5 "final" session ran)
# A session is one gpurun call chaining subcommands with &&, e.g.
#   gpurun -- 'bash scripts/gpu.sh tests r6a && bash scripts/gpu.sh envab r6a "X=1" "X=0"'
# (round 5's 58 one-off scripts/r5*_session.sh were exactly such chains; they are in the git history.)
# (Round 4 replaced the per-experiment scripts/gpu_*.sh launchers that older profiles/ notes name with these modes;
#  their exact commands are in the git history.)
# Every GPU step runs under its own time limit and the script stops at the first failure.
set -o pipefail
ROOT="${GRAFT_REPO_ROOT:-/root/repo}"
OUT="$ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
WHAT=${1:-bench}
TAG=${2:-x}
shift 2 2>/dev/null
fail() { echo "$1 failed"; tail -30 "$2"; exit 1; }

prof_one() {   # name script args...
  local name=$1; shift
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/prof_${name}_$TAG" -o run \
      --output-format csv -- python3 "$@") > "$OUT/prof_${name}_$TAG.log" 2>&1 || fail "prof $name" "$OUT/prof_${name}_$TAG.log"
  echo "prof $name ok"
}

case "$WHAT" in
  tests)
    cd "$ROOT"
    timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread "$@" \
        > "$OUT/pytest_gpu_$TAG.log" 2>&1
    rc=$?
    tail -15 "$OUT/pytest_gpu_$TAG.log"
    exit $rc ;;
  bench)
    cd "$ROOT"
    for i in 1 2 3; do
      timeout -k 10 300 python bench.py "$@" > "$OUT/bench_${TAG}_$i.log" 2>&1 || fail "bench $i" "$OUT/bench_${TAG}_$i.log"
      tail -1 "$OUT/bench_${TAG}_$i.log"
    done ;;
  prof)
    prof_one resnet "$ROOT/bench.py" --steps 5 --warmup 3 --bert 0 "$@"
    prof_one bert "$ROOT/bench/bert_bench.py" --steps 5 --warmup 3
    cd "$ROOT" && python scripts/step_breakdown.py "$OUT/prof_resnet_$TAG" --calls > "$OUT/summary_resnet_$TAG.txt" 2>&1
    python scripts/step_breakdown.py "$OUT/prof_bert_$TAG" --calls > "$OUT/summary_bert_$TAG.txt" 2>&1
    head -30 "$OUT/summary_resnet_$TAG.txt" ;;
  profr)
    prof_one resnet "$ROOT/bench.py" --steps 5 --warmup 3 --bert 0 "$@"
    cd "$ROOT" && python scripts/step_breakdown.py "$OUT/prof_resnet_$TAG" --calls > "$OUT/summary_resnet_$TAG.txt" 2>&1
    head -40 "$OUT/summary_resnet_$TAG.txt" ;;
  pmc)
    P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CU_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"
    P2="FETCH_SIZE GRBM_GUI_ACTIVE"
    P3="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
    i=0
    for P in "$P1" "$P2" "$P3"; do
      i=$((i+1))
      (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace -d "$OUT/pmcr_${TAG}_p$i" -o run \
          --output-format csv -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --hip_graph ${PMC_GRAPH:-1} --bert 0) \
          > "$OUT/pmcr_${TAG}_p$i.log" 2>&1 || fail "resnet pmc $i" "$OUT/pmcr_${TAG}_p$i.log"
      (cd /tmp && timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace -d "$OUT/pmcb_${TAG}_p$i" -o run \
          --output-format csv -- python3 "$ROOT/bench/bert_bench.py" --steps 2 --warmup 1 --hip_graph ${PMC_GRAPH:-1}) \
          > "$OUT/pmcb_${TAG}_p$i.log" 2>&1 || fail "bert pmc $i" "$OUT/pmcb_${TAG}_p$i.log"
      echo "pmc pass $i ok"
    done ;;
  envab)
    A=$1; B=$2; STEPS=${3:-30}
    cd "$ROOT"
    for i in 1 2 3; do
      for arm in A B; do
        if [ $arm = A ]; then E=$A; else E=$B; fi
        env $E timeout -k 10 300 python bench.py --steps $STEPS --warmup 5 --bert 0 > "$OUT/ab_${TAG}_${arm}_$i.log" 2>&1 \
          || fail "ab $arm $i" "$OUT/ab_${TAG}_${arm}_$i.log"
        echo "$arm($E) $(tail -1 "$OUT/ab_${TAG}_${arm}_$i.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
      done
    done ;;
  bertab)
    A=$1; B=$2; STEPS=${3:-30}
    cd "$ROOT"
    for i in 1 2 3; do
      for arm in A B; do
        if [ $arm = A ]; then E=$A; else E=$B; fi
        env $E timeout -k 10 300 python bench/bert_bench.py --steps $STEPS --warmup 5 > "$OUT/bab_${TAG}_${arm}_$i.log" 2>&1 \
          || fail "bert ab $arm $i" "$OUT/bab_${TAG}_${arm}_$i.log"
        echo "$arm($E) $(tail -1 "$OUT/bab_${TAG}_${arm}_$i.log" | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
      done
    done ;;
  rehearse2)
    cd "$ROOT"
    MDTF_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --bert 0 \
        > "$OUT/rehearse2_$TAG.json" 2> "$OUT/rehearse2_$TAG.err" || fail "rehearsal" "$OUT/rehearse2_$TAG.err"
    tail -1 "$OUT/rehearse2_$TAG.json" | cut -c1-400
    MDTF_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --bert 0 --mode sharded \
        --comm_dtype bf16 > "$OUT/rehearse2s_$TAG.json" 2> "$OUT/rehearse2s_$TAG.err" || fail "sharded rehearsal" "$OUT/rehearse2s_$TAG.err"
    tail -1 "$OUT/rehearse2s_$TAG.json" | cut -c1-400 ;;
  pmcpy)   # gpu.sh pmcpy TAG "COUNTERS" script.py [args]: one counter pass over a python script
    C=$1; S=$2; shift 2
    (cd /tmp && timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d "$OUT/pmcpy_$TAG" -o run \
        --output-format csv -- python3 "$ROOT/$S" "$@") > "$OUT/pmcpy_$TAG.log" 2>&1 || fail "pmc $S" "$OUT/pmcpy_$TAG.log"
    echo "pmcpy $TAG ok" ;;
  py)
    cd "$ROOT"
    S=$1; shift
    timeout -k 10 600 python -u "$S" "$@" > "$OUT/py_$TAG.log" 2>&1 || fail "py $S" "$OUT/py_$TAG.log"
    tail -40 "$OUT/py_$TAG.log" ;;
  final)
    bash "$ROOT/scripts/gpu.sh" tests "$TAG" && \
    bash "$ROOT/scripts/gpu.sh" bench "$TAG" --steps 30 --warmup 5 && \
    bash "$ROOT/scripts/gpu.sh" prof "$TAG" > /dev/null && echo "prof ok" ;;
  *)
    echo "unknown: $WHAT"; exit 2 ;;
esac
