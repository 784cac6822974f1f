#!/usr/bin/env python
"""BERT pre-training throughput (sequences/sec, whole job) — BASELINE config 4.

BERT-base (or --size large), sequence length 128, 20 masked predictions,
synthetic token data, random-init weights, fused AdamWeightDecay; one process
per GPU (torchrun) with bucketed RCCL gradient all-reduce.  ``--stock`` runs
the comparator: a plain torch.nn BERT with scaled_dot_product_attention,
autocast bf16, torch AdamW (fused=False/foreach) and DDP.
"""
import argparse
import json
import math
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--seq", type=int, default=128)
    p.add_argument("--size", default="base")
    p.add_argument("--stock", action="store_true")
    p.add_argument("--mode", default="allreduce", choices=["allreduce", "sharded"])
    p.add_argument("--hip_graph", type=int, default=1, help="capture the mdtf training step in a hipGraph")
    p.add_argument("--comm_dtype", default=None, choices=["fp32", "bf16"], help="gradient wire dtype")
    p.add_argument("--bucket_mb", type=int, default=None, help="gradient bucket MiB")
    p.add_argument("--trace_ops", default=None,
                   help="after the warm-up, profile one step with Python stacks (use --hip_graph 0) into this dir")
    return p.parse_args()


class StockLayer(nn.Module):
    def __init__(self, H, nh, I):
        super().__init__()
        self.nh = nh
        self.qkv = nn.Linear(H, 3 * H)
        self.o = nn.Linear(H, H)
        self.ln1 = nn.LayerNorm(H, eps=1e-12)
        self.i = nn.Linear(H, I)
        self.out = nn.Linear(I, H)
        self.ln2 = nn.LayerNorm(H, eps=1e-12)

    def forward(self, x, mask):
        B, S, H = x.shape
        q, k, v = self.qkv(x).view(B, S, 3, self.nh, H // self.nh).permute(2, 0, 3, 1, 4)
        a = F.scaled_dot_product_attention(q, k, v, attn_mask=mask, dropout_p=0.1)
        a = a.transpose(1, 2).reshape(B, S, H)
        x = self.ln1(x + F.dropout(self.o(a), 0.1))
        return self.ln2(x + F.dropout(self.out(F.gelu(self.i(x), approximate="tanh")), 0.1))


class StockBert(nn.Module):
    def __init__(self, V=30522, H=768, L=12, nh=12, I=3072, S=512):
        super().__init__()
        self.word = nn.Embedding(V, H)
        self.pos = nn.Embedding(S, H)
        self.typ = nn.Embedding(2, H)
        self.ln = nn.LayerNorm(H, eps=1e-12)
        self.layers = nn.ModuleList([StockLayer(H, nh, I) for _ in range(L)])
        self.pool = nn.Linear(H, H)
        self.tr = nn.Linear(H, H)
        self.tln = nn.LayerNorm(H, eps=1e-12)
        self.obias = nn.Parameter(torch.zeros(V))
        self.nsp = nn.Linear(H, 2)

    def forward(self, ids, types, mask, positions):
        B, S = ids.shape
        x = self.word(ids) + self.pos(torch.arange(S, device=ids.device)) + self.typ(types)
        x = F.dropout(self.ln(x), 0.1)
        am = ((1.0 - mask.to(x.dtype)) * -10000.0)[:, None, None, :]
        for l in self.layers:
            x = l(x, am)
        pooled = torch.tanh(self.pool(x[:, 0]))
        idx = (positions + torch.arange(B, device=ids.device)[:, None] * S).reshape(-1)
        h = self.tln(F.gelu(self.tr(x.reshape(B * S, -1).index_select(0, idx)), approximate="tanh"))
        return h @ self.word.weight.t() + self.obias, self.nsp(pooled)


# stock PyTorch-ROCm comparator (this script with --stock: SDPA flash attention, torch AdamW, DDP) on one
# MI355X at the default config (BERT-base, seq 128, batch 64): README / profiles/rocprof_bert_base_stock_r1_summary.txt
STOCK_SEQ128_PER_GPU = 3319.0


def main():
    args = parse()
    graph_op = None                  # the mdtf train op (its StepGraph says whether replays happened)
    from mdtf.utils.launch import ensure_ranks
    ensure_ranks(args.gpus, os.path.abspath(__file__))     # --gpus N: N ranks or a non-zero exit
    distributed = int(os.environ.get("WORLD_SIZE", "1")) > 1
    if distributed:
        from mdtf.cluster import Server
        server = Server.from_env()
        rank, world = dist.get_rank(), dist.get_world_size()
        pg = server.worker_group
    else:
        server, rank, world, pg = None, 0, 1, None
    lr = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = torch.cuda.is_available()
    # the server's device: one per local rank, or shared when an MDTF_DIST_BACKEND=gloo rehearsal runs more ranks
    # than there are GPUs (as bench.py); cpu: gloo rehearsal of the launch
    dev = (server.device() if server is not None else torch.device("cuda", lr)) if gpu else torch.device("cpu")
    if gpu:
        torch.cuda.set_device(dev)
    if args.stock and not gpu:
        raise SystemExit("--stock needs a GPU")
    from mdtf.models import Bert, BertPretrainingLoss, SyntheticBertLoader
    from mdtf.models.bert import CONFIGS
    P = 20
    if args.stock:
        cfg = CONFIGS[args.size]
        model = StockBert(H=cfg["hidden"], L=cfg["layers"], nh=cfg["heads"], I=cfg["intermediate"]).to(dev)
        if distributed:
            model = nn.parallel.DistributedDataParallel(model, device_ids=[lr], bucket_cap_mb=32)
        opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=0.01, foreach=True)
        ld = SyntheticBertLoader(args.seq, P, seed=rank)
        ld.batch_size = args.batch
        from mdtf.train import variables as V
        V.get_store().device = dev
        raw, gt = ld._make()
        S = args.seq
        ids, types, mask, pos = raw[:, :S], raw[:, S:2 * S], raw[:, 2 * S:3 * S], raw[:, 3 * S:3 * S + P]

        def step():
            opt.zero_grad(set_to_none=True)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                mlm, nsp = model(ids, types, mask, pos)
                loss = F.cross_entropy(mlm.float(), gt[:, :P].reshape(-1)) + F.cross_entropy(nsp.float(), gt[:, P])
            loss.backward()
            opt.step()
            return loss
        run = step
    else:
        import mdtf
        from mdtf.runtime import Net, Tower
        from mdtf.train import variables as V
        store = V.get_store()
        store.device = dev
        store.compute_dtype = torch.bfloat16 if gpu else None
        ld = SyntheticBertLoader(args.seq, P, seed=rank)
        ld.batch_size = args.batch
        raw, gt = ld.load_train_batch()
        base = mdtf.train.AdamWeightDecayOptimizer(1e-4, weight_decay_rate=0.01)
        tg = []
        tower = Tower(Net(Bert(args.size, seq_len=args.seq, max_predictions=P)), "tower_0/", tg, raw, gt,
                      BertPretrainingLoss(P), base, batch_size=args.batch)
        _, loss_h, _ = tower.process()
        opt = mdtf.train.SyncReplicasOptimizer(base, world, world, hip_graph=bool(args.hip_graph) and gpu,
                                               mode=args.mode, comm_dtype=args.comm_dtype,
                                               bucket_bytes=(args.bucket_mb << 20) if args.bucket_mb else None)
        op = opt.apply_gradients(Tower.average_gradients(tg), global_step=mdtf.train.get_or_create_global_step())
        graph_op = op
        sess = mdtf.train.MonitoredTrainingSession(is_chief=rank == 0, log_step_count_steps=0, server=server)

        def run():
            sess.run(op)
    def sync():
        if gpu:
            torch.cuda.synchronize()

    for _ in range(args.warmup):
        run()
    sync()
    if args.trace_ops and rank == 0:
        from torch.profiler import ProfilerActivity, profile
        with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True,
                     with_stack=True) as prof:
            run()
            torch.cuda.synchronize()
        os.makedirs(args.trace_ops, exist_ok=True)
        with open(os.path.join(args.trace_ops, "ops_by_shape.txt"), "w") as f:
            f.write(prof.key_averages(group_by_input_shape=True).table(sort_by="self_cuda_time_total", row_limit=80,
                                                                       max_name_column_width=40,
                                                                       max_shapes_column_width=80))
        with open(os.path.join(args.trace_ops, "ops_by_stack.txt"), "w") as f:
            f.write(prof.key_averages(group_by_stack_n=6).table(sort_by="self_cuda_time_total", row_limit=60,
                                                                 max_name_column_width=40))
        with open(os.path.join(args.trace_ops, "ops_parents.txt"), "w") as f:
            for e in prof.events():
                if e.name in ("aten::add_", "aten::add", "aten::fill_", "aten::copy_", "aten::cat"):
                    chain, p = [], e.cpu_parent
                    while p is not None and len(chain) < 4:
                        chain.append(p.name)
                        p = p.cpu_parent
                    f.write("%s %s <- %s\n" % (e.name, str(e.input_shapes)[:80], " < ".join(chain)))
    if world > 1:
        dist.barrier(group=pg)
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run()
    sync()
    if world > 1:
        dist.barrier(group=pg)
    el = torch.tensor([time.perf_counter() - t0], device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX, group=pg)
    el = float(el)
    if rank == 0:
        sps = world * args.batch * args.steps / el
        print(json.dumps({"metric": "sequences/sec BERT-%s pretraining seq%d" % (args.size, args.seq),
                          "value": round(sps, 2), "unit": "sequences/sec", "n_gpus": world,
                          "per_gpu_sequences_per_sec": round(sps / world, 2), "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": round(1000 * el / args.steps, 3),
                          "higher_is_better": True, "scaling": "weak",
                          "vs_baseline": (round(sps / (STOCK_SEQ128_PER_GPU * world), 4)
                                          if (args.size, args.seq, args.batch) == ("base", 128, 64) and not args.stock
                                          else None),
                          "baseline": "stock PyTorch-ROCm comparator, %.0f seq/s/GPU x %d" % (
                              STOCK_SEQ128_PER_GPU, world),
                          "impl": "stock-pytorch" if args.stock else "mdtf",
                          # a captured step really replayed (gloo rehearsals / a rejected capture run eagerly)
                          "hip_graph": (not args.stock and gpu
                                        and bool(getattr(getattr(graph_op, "graph", None), "replays", 0))),
                          "dtype": "bf16" if gpu else "fp32",
                          "data": "synthetic (random token ids, random-init weights)",
                          "config": {"model": "bert-%s" % args.size, "global_batch": world * args.batch,
                                     "per_gpu_batch": args.batch, "seq_len": args.seq,
                                     "parallelism": "dp%d" % world,
                                     "grad_sync": "ddp" if args.stock else args.mode,
                                     "optimizer": "torch AdamW" if args.stock else "AdamWeightDecay (fused)"}}),
              flush=True)
    if not args.stock:
        sess.close()
    if distributed:
        from mdtf.train import step as S_
        S_.release_graphs()
        dist.barrier(group=pg)
        server.shutdown()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
