cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && \
for arm in "allreduce bf16 1" "sharded bf16 1" "sharded bf16 0" "allreduce fp32 1" "sharded fp32 1"; do
  set -- $arm
  MDTF_GLOO_RS_AR=$3 MDTF_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --bert 0 --mode $1 --comm_dtype $2 > gpurun_out/reh_r5z_$1_$2_$3.json 2> gpurun_out/reh_r5z_$1_$2_$3.err || { echo "rehearsal $arm failed"; tail -20 gpurun_out/reh_r5z_$1_$2_$3.err; exit 1; }
  echo "$arm $(tail -1 gpurun_out/reh_r5z_$1_$2_$3.json | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
