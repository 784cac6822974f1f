#!/usr/bin/env python
"""Headline benchmark: ResNet-50 v1.5 sync-SGD training throughput (images/sec, whole job).

BASELINE.json metric: "images/sec (whole node) ResNet-50 sync-SGD at 1/2/4/8
MI355X; scaling efficiency".  One process per GPU (torchrun); each step is a
full training step through the framework engine: forward + backward of
ResNet-50 (bf16 compute, fp32 master weights) on a synthetic ImageNet-shaped
batch (224x224x3, 1000 classes, random-init weights), bucketed RCCL
gradient reduction overlapped with backward, fused momentum-SGD update.

    python bench.py --gpus 1 --steps 20 --warmup 5
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 20 --warmup 5

Timing: W untimed warmup steps, then barrier + device sync, K timed steps,
barrier + device sync; the elapsed time is the MAX over ranks; rank 0 prints
one JSON line.  ``value`` = N * per_gpu_batch * K / elapsed (weak scaling).
"""
import argparse
import json
import os
import sys
import time

# The reference publishes no numbers; its comparator is stock PyTorch-ROCm on the
# same MI355X (MIOpen conv/BN, torch DDP over RCCL, torch SGD, channels-last autocast bf16),
# measured with bench/stock_pytorch.py at this config on 1 GPU: 5966.38 images/sec
# (profiles/rocprof_resnet50_stock_torch_ops_r1.md).  vs_baseline divides by that rate x N
# (ideal linear scaling of the comparator, i.e. a conservative ratio for N > 1).
BASELINE_IMAGES_PER_SEC_PER_GPU = 5966.38


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    p.add_argument("--depth", type=int, default=50)
    p.add_argument("--mode", default="allreduce", choices=["allreduce", "sharded"])
    p.add_argument("--kernels", default=None, help="native|torch (MDTF_KERNELS)")
    p.add_argument("--bucket_mb", type=int, default=None, help="gradient bucket MiB (default MDTF_BUCKET_MB or 32)")
    p.add_argument("--comm_dtype", default=None, choices=["fp32", "bf16"],
                   help="gradient wire dtype of the RCCL reductions (default MDTF_COMM_DTYPE or fp32)")
    p.add_argument("--profile_dir", default=None)
    p.add_argument("--hip_graph", type=int, default=1,
                   help="1: capture the whole training step in a hipGraph after 2 eager steps (mdtf.train.graph)")
    p.add_argument("--image_size", type=int, default=224, help="image side (CPU tests of the launch path use 32-64)")
    p.add_argument("--ref_rate", type=float, default=None,
                   help="per-GPU images/sec of the N=1 run of this config, for scaling_efficiency (default: the rate the "
                        "last N=1 run of the same config cached in .bench_n1_rate.json)")
    p.add_argument("--bert", type=int, default=-1,
                   help="also measure BERT-base (bench/bert_bench.py, a child process run before the ResNet job) and "
                        "attach it under extra.bert_base; -1: on for the default 1-GPU run")
    return p.parse_args()


def _bert_child(args):
    """BASELINE config 4 on 1 GPU, measured by bench/bert_bench.py in a child process (before this process
    touches the GPU) so the driver's bench run also records it; None if skipped or failed."""
    import subprocess
    want = args.bert if args.bert >= 0 else int(args.gpus == 1 and args.image_size == 224
                                                   and "RANK" not in os.environ)
    if not want:
        return None
    here = os.path.dirname(os.path.abspath(__file__))
    cmd = [sys.executable, os.path.join(here, "bench", "bert_bench.py"), "--steps", "20", "--warmup", "5"]
    try:
        out = subprocess.run(cmd, capture_output=True, text=True, timeout=400)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")][-1]
        rec = json.loads(line)
        return {k: rec.get(k) for k in ("metric", "value", "unit", "ms_per_step", "steps", "warmup", "vs_baseline",
                                        "baseline", "config") if k in rec}
    except Exception as e:  # noqa: BLE001 - the ResNet measurement must not depend on it
        return {"error": "%s: %s" % (type(e).__name__, str(e)[:200])}


def _ensure_ranks(args):
    """--gpus N is honoured: under torchrun WORLD_SIZE must equal N, otherwise N ranks are spawned
    (mdtf/utils/launch.py; loaded by path so nothing imports torch or touches the GPU first)."""
    import importlib.util
    here = os.path.dirname(os.path.abspath(__file__))
    spec = importlib.util.spec_from_file_location("_mdtf_launch", os.path.join(here, "mdtf", "utils", "launch.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    mod.ensure_ranks(args.gpus, os.path.abspath(__file__))


def main():
    args = parse()
    _ensure_ranks(args)
    bert = _bert_child(args)
    if args.kernels:
        os.environ["MDTF_KERNELS"] = args.kernels
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import mdtf
    from mdtf.cluster import Server
    from mdtf.data.loaders import SyntheticDataLoader
    from mdtf.models import ResNet, SoftmaxCrossEntropyLoss
    from mdtf.runtime import Net, Tower
    from mdtf.train import variables as V
    from mdtf.train import step as S

    distributed = "RANK" in os.environ and int(os.environ.get("WORLD_SIZE", "1")) > 1
    if distributed:
        server = Server.from_env()
        world, rank = dist.get_world_size(), dist.get_rank()
        dev = server.device()
        pg = server.worker_group
    else:
        server, world, rank, pg = None, 1, 0, None
        dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
    store = V.get_store()
    store.device = dev
    store.compute_dtype = torch.bfloat16 if dev.type == "cuda" else None
    store.generator.manual_seed(1234)

    loader = SyntheticDataLoader(shape=(args.image_size, args.image_size, 3), num_classes=1000,
                                 dtype=torch.bfloat16 if dev.type == "cuda" else torch.float32, seed=rank)
    loader.batch_size = args.batch
    raw, gt = loader.load_train_batch()
    base = mdtf.train.MomentumOptimizer(0.1 * args.batch * world / 256.0, momentum=0.9, weight_decay=5e-5)
    gs = mdtf.train.get_or_create_global_step()
    tower_grads = []
    tower = Tower(Net(ResNet(args.depth)), "tower_0/", tower_grads, raw, gt, SoftmaxCrossEntropyLoss(), base,
                  batch_size=args.batch)
    _, loss, _ = tower.process()
    opt = mdtf.train.SyncReplicasOptimizer(base, replicas_to_aggregate=world, total_num_replicas=world,
                                           mode=args.mode, hip_graph=bool(args.hip_graph),
                                           bucket_bytes=(args.bucket_mb << 20) if args.bucket_mb else None,
                                           comm_dtype=args.comm_dtype)
    train_op = opt.apply_gradients(Tower.average_gradients(tower_grads), global_step=gs)
    sess = mdtf.train.MonitoredTrainingSession(is_chief=(rank == 0), checkpoint_dir=None, log_step_count_steps=0,
                                               server=server)

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier(group=pg)

    for _ in range(args.warmup):
        sess.run(train_op)
    lv = sess.run(loss)
    sync()
    prof = None
    if args.profile_dir and rank == 0:
        prof = torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU,
                                                  torch.profiler.ProfilerActivity.CUDA])
        prof.__enter__()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        sess.run(train_op)
    sync()
    elapsed = time.perf_counter() - t0
    if prof is not None:
        prof.__exit__(None, None, None)
        os.makedirs(args.profile_dir, exist_ok=True)
        with open(os.path.join(args.profile_dir, "torch_profile.txt"), "w") as f:
            f.write(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=80))
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev if dev.type == "cuda" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=pg)
    elapsed = float(t.item())
    # the communicator's own rank count (a SUM all-reduce of ones over the training group), so a scaling record
    # shows that RCCL -- not a fallback -- saw every rank
    comm = {"backend": None, "ranks_in_collective": 1}
    if distributed and dist.is_initialized():
        one = torch.ones(1, dtype=torch.float32, device=dev if dev.type == "cuda" else "cpu")
        dist.all_reduce(one, group=pg)
        comm = {"backend": str(dist.get_backend(pg)), "ranks_in_collective": int(round(float(one.item())))}
    final_loss = float(sess.run(loss))
    if rank == 0:
        ips = world * args.batch * args.steps / elapsed
        base_ips = BASELINE_IMAGES_PER_SEC_PER_GPU
        rec = {
            "metric": "images/sec (whole node) ResNet-50 sync-SGD at 1/2/4/8 MI355X; scaling efficiency",
            "value": round(ips, 2), "unit": "images/sec", "n_gpus": world,
            "per_gpu_images_per_sec": round(ips / world, 2), "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(1000.0 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": "weak",
            "vs_baseline": round(ips / (base_ips * world), 4) if base_ips else None,
            "baseline": "stock PyTorch-ROCm comparator, %.2f img/s/GPU x %d" % (base_ips, world) if base_ips else None,
            "dtype": "bf16" if dev.type == "cuda" else "fp32",
            "data": "synthetic (random %dx%dx3 NHWC images, random labels; random-init weights)" % (
                args.image_size, args.image_size),
            "config": {"model": "resnet%d_v1.5" % args.depth, "global_batch": args.batch * world, "seq_len": None,
                       "per_gpu_batch": args.batch, "image_size": args.image_size, "parallelism": "dp%d" % world,
                       "grad_sync": args.mode,
                       "comm_dtype": "bf16" if str(opt.comm_dtype or os.environ.get("MDTF_COMM_DTYPE", "fp32")).startswith("bf") else "fp32",
                       "optimizer": "momentum-sgd (fused)",
                       "kernels": os.environ.get("MDTF_KERNELS", "native"),
                       # whether the step really replayed a captured graph (gloo rehearsals and a rejected
                       # capture run eagerly)
                       "hip_graph": bool(getattr(getattr(train_op, "graph", None), "replays", 0))},
            "loss_first": float(lv), "loss_last": final_loss, "comm": comm,
        }
        # scaling efficiency = rate(N) / (N x rate(1)) against this config's N=1 rate (--ref_rate, or the rate
        # the last N=1 run cached next to this file)
        key = "resnet%d/b%d/i%d/%s/%s" % (args.depth, args.batch, args.image_size, args.mode,
                                          rec["config"]["comm_dtype"])
        cache = os.path.join(os.path.dirname(os.path.abspath(__file__)), ".bench_n1_rate.json")
        try:
            cached = json.load(open(cache)) if os.path.exists(cache) else {}
        except ValueError:
            cached = {}
        if world == 1:
            cached[key] = ips
            try:
                with open(cache, "w") as f:
                    json.dump(cached, f)
            except OSError:
                pass
        ref = args.ref_rate or cached.get(key)
        rec["scaling_efficiency"] = round(ips / (world * ref), 4) if ref else None
        rec["scaling_ref_rate_per_gpu"] = round(ref, 2) if ref else None
        if bert is not None:
            rec["extra"] = {"bert_base": bert}
        print(json.dumps(rec), flush=True)
    sess.close()
    if distributed:
        # the captured step graph holds RCCL collectives: sess.close() released it; now the communicator
        S.release_graphs()
        dist.barrier(group=pg)
        server.shutdown()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
