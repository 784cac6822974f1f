# per-GPU batch / depth / size sweep of both benches on one MI355X (each step under its own limit; stop at the
# first abort, fault or time limit; a plain Python error (rc 1) is recorded and the sweep goes on)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
run() {   # tag cmd...
  local tag=$1; shift
  timeout -k 10 300 "$@" > gpurun_out/sweep_$tag.log 2>&1
  local rc=$?
  echo "$tag rc=$rc $(tail -1 gpurun_out/sweep_$tag.log | cut -c1-200)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
run rn50_b128 python bench.py --bert 0 --batch 128 --steps 30 --warmup 5
run rn50_b384 python bench.py --bert 0 --batch 384 --steps 30 --warmup 5
run rn50_b512 python bench.py --bert 0 --batch 512 --steps 30 --warmup 5
run rn101_b256 python bench.py --bert 0 --depth 101 --steps 20 --warmup 5
run rn152_b256 python bench.py --bert 0 --depth 152 --steps 20 --warmup 5
run bert_b32 python bench/bert_bench.py --batch 32 --steps 30 --warmup 5
run bert_b128 python bench/bert_bench.py --batch 128 --steps 30 --warmup 5
run bert_b256 python bench/bert_bench.py --batch 256 --steps 20 --warmup 5
run bertL_b32 python bench/bert_bench.py --size large --batch 32 --steps 20 --warmup 5
