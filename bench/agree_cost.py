#!/usr/bin/env python
"""Cost of the per-step recovery agreement of multi-replica sessions (``MonitoredSession._agree``: one 4-byte
gloo all-reduce(MAX) per ``run``), at N ranks on one host.

    python bench/agree_cost.py --ranks 8 --iters 2000 [--out profiles/agree_cost_r4.json]

Each rank calls the session's own ``_agree`` (a MonitoredSession shell bound to a gloo group) ``iters`` times;
the report is the per-call latency (median / p90 / max over ranks of each rank's median) and its share of the
ResNet-50 step at the measured 1-GPU step time."""
import argparse
import json
import os
import socket
import statistics
import sys
import time

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


STEP_S = 0.0228


def _rank(rank, world, port, iters, q, step_s=0.0228):
    global STEP_S
    STEP_S = step_s
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from mdtf.train.session import MonitoredSession
    sess = MonitoredSession.__new__(MonitoredSession)      # only the agreement machinery is exercised
    sess._agree_pg = MonitoredSession._agreement_group(dist.group.WORLD)
    sess._agree_buf = None
    for _ in range(50):
        sess._agree(0)
    lat = []
    for i in range(iters):
        t0 = time.perf_counter()
        sess._agree(0)
        lat.append(time.perf_counter() - t0)
    lat.sort()
    # async form (the session default): post at the boundary, the step runs (a sleep of the step time here),
    # wait at the next boundary; only the post and the wait cost host time on the step's critical path
    sess._agree_work = None
    sess.agreements = 0
    alat = []
    for i in range(min(iters, 200)):
        t0 = time.perf_counter()
        if sess._agree_work is not None:
            sess._agree_result()
        sess._agree_post(0)
        alat.append(time.perf_counter() - t0)
        time.sleep(STEP_S)
    sess._agree_result()
    alat.sort()
    q.put({"rank": rank, "median_us": 1e6 * lat[len(lat) // 2], "p90_us": 1e6 * lat[int(0.9 * len(lat))],
           "max_us": 1e6 * lat[-1], "async_median_us": 1e6 * alat[len(alat) // 2],
           "async_p90_us": 1e6 * alat[int(0.9 * len(alat))]})
    dist.barrier()
    dist.destroy_process_group()


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--ranks", type=int, default=8)
    p.add_argument("--iters", type=int, default=2000)
    p.add_argument("--step_ms", type=float, default=22.8, help="training step time to price the agreement against")
    p.add_argument("--out", default=None)
    a = p.parse_args()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, a.ranks, port, a.iters, q, a.step_ms / 1000.0)) for r in range(a.ranks)]
    for pr in procs:
        pr.start()
    res = [q.get(timeout=600) for _ in procs]
    for pr in procs:
        pr.join()
    med = max(r["median_us"] for r in res)
    rec = {"what": "MonitoredSession agreement: 4-byte gloo all-reduce(MAX) per run, host CPU ranks; sync = blocking round trip, async = post at one boundary + wait at the next (the default, MDTF_AGREE=async)",
           "ranks": a.ranks, "iters": a.iters, "median_us_worst_rank": round(med, 1),
           "p90_us_worst_rank": round(max(r["p90_us"] for r in res), 1),
           "median_us_per_rank": [round(r["median_us"], 1) for r in sorted(res, key=lambda r: r["rank"])],
           "step_ms": a.step_ms, "share_of_step_pct": round(100.0 * med / (1000.0 * a.step_ms), 3),
           "async_post_plus_wait_us_worst_rank": round(max(r["async_median_us"] for r in res), 1),
           "async_p90_us_worst_rank": round(max(r["async_p90_us"] for r in res), 1),
           "async_share_of_step_pct": round(100.0 * max(r["async_median_us"] for r in res) / (1000.0 * a.step_ms),
                                            3),
           "cpus": os.cpu_count()}
    print(json.dumps(rec))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
