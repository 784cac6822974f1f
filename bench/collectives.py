#!/usr/bin/env python
"""RCCL collective bandwidth over xGMI at gradient-bucket sizes (pick the bucket size).

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench/collectives.py

For every size (4..256 MiB by default) and collective (all_reduce, reduce_scatter, all_gather;
fp32 and bf16) it times ``--iters`` launches after ``--warmup`` and prints one JSON line per
case: algorithm bandwidth (bytes / time) and bus bandwidth (the nccl-tests convention:
all_reduce x 2(N-1)/N, reduce_scatter / all_gather x (N-1)/N), the max over ranks.
"""
import argparse
import json
import os
import time

import torch
import torch.distributed as dist


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--sizes_mb", default="4,8,16,32,64,128,256")
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--dtypes", default="float32,bfloat16")
    a = p.parse_args()
    cuda = torch.cuda.is_available()
    backend = "nccl" if cuda else "gloo"
    if cuda:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(backend)
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda") if cuda else torch.device("cpu")
    for dt_name in a.dtypes.split(","):
        dt = getattr(torch, dt_name)
        for mb in [int(x) for x in a.sizes_mb.split(",")]:
            n = mb * (1 << 20) // torch.tensor([], dtype=dt).element_size()
            n -= n % world
            buf = torch.ones(n, dtype=dt, device=dev)
            shard = torch.empty(n // world, dtype=dt, device=dev)
            for name in ("all_reduce", "reduce_scatter", "all_gather"):
                def op():
                    if name == "all_reduce":
                        dist.all_reduce(buf)
                    elif name == "reduce_scatter":
                        dist.reduce_scatter_tensor(shard, buf)
                    else:
                        dist.all_gather_into_tensor(buf, shard)
                for _ in range(a.warmup):
                    op()
                if cuda:
                    torch.cuda.synchronize()
                dist.barrier()
                t0 = time.perf_counter()
                for _ in range(a.iters):
                    op()
                if cuda:
                    torch.cuda.synchronize()
                el = torch.tensor([(time.perf_counter() - t0) / a.iters], device=dev)
                dist.all_reduce(el, op=dist.ReduceOp.MAX)
                t = float(el)
                nbytes = n * buf.element_size()
                factor = 2.0 * (world - 1) / world if name == "all_reduce" else (world - 1) / world
                if rank == 0:
                    print(json.dumps({"collective": name, "dtype": dt_name, "bytes": nbytes, "n_ranks": world,
                                      "us": round(t * 1e6, 1), "algbw_GBps": round(nbytes / t / 1e9, 2),
                                      "busbw_GBps": round(nbytes / t / 1e9 * factor, 2)}), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
