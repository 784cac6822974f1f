#!/usr/bin/env python
"""Dense GEMMs of BERT-base on the weight-stationary streamed kernel (csrc/conv_ws.hip, run as a 1x1 convolution
over M = 8192 "pixels" viewed as [M/64, 8, 8, K]) vs hipBLASLt, both timed inside captured graphs.  Forward
y = x W (the kernel takes W^T, K-contiguous) and data gradient dx = dy W^T (W as is), every candidate tile."""
import itertools
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdtf.ops import conv as C  # noqa: E402
from mdtf.ops import tunable  # noqa: E402

M = 8192
FWD = [(768, 2304), (768, 768), (768, 3072)]          # (K, N): qkv, attention-out, FFN-in  (ws: K <= 1280)
DGRAD = [(768, 768), (3072, 768)]                      # (K, N): attention-out, FFN-out      (ws: N <= 1280)
TILES = [(tp, nw, cg, d) for tp, nw, cg, d in itertools.product((2, 4), (4, 8), (1, 2, 4), (3, 4, 6))]


def gtime(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) / reps)
    return statistics.median(ts)


def try_tiles(run, ref):
    res = {}
    for t in TILES:
        try:
            y = run(t)
            torch.cuda.synchronize()
        except RuntimeError:
            continue
        err = ((y.float() - ref).norm() / ref.norm()).item()
        if err > 2e-2:
            res[t] = ("bad", err)
            continue
        res[t] = gtime(lambda: run(t))
    return res


def main():
    dev = torch.device("cuda")
    tunable.ensure(dev)
    for K, N in FWD:
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(K, N, device=dev) * 0.03).bfloat16()
        wt = w.t().contiguous()
        ref = torch.mm(x, w).float()
        t_lib = gtime(lambda: torch.mm(x, w))
        x4 = x.view(M // 64, 8, 8, K)
        res = try_tiles(lambda t: C.ws_fwd(x4, wt, 1, 1, (8, 8), (1, 1), (0, 0, 0, 0), (1, 1), t).view(M, N), ref)
        ok = {t: v for t, v in res.items() if not isinstance(v, tuple)}
        best = min(ok, key=ok.get) if ok else None
        print(json.dumps({"pass": "fwd", "M": M, "K": K, "N": N, "lib_ms": round(t_lib, 4),
                          "ws_ms": round(ok[best], 4) if best else None, "tile": best,
                          "bad": [t for t, v in res.items() if isinstance(v, tuple)],
                          "all": {"%d/%d/%d/%d" % t: round(v, 4) for t, v in sorted(ok.items(), key=lambda kv: kv[1])[:6]}}),
              flush=True)
    for K, N in DGRAD:
        dy = torch.randn(M, N, device=dev).bfloat16()
        w = (torch.randn(K, N, device=dev) * 0.03).bfloat16()
        ref = torch.mm(dy, w.t()).float()
        t_lib = gtime(lambda: torch.mm(dy, w.t()))
        dy4 = dy.view(M // 64, 8, 8, N)
        w4 = w.view(1, 1, K, N)
        res = try_tiles(lambda t: C.ws_dgrad(dy4, w4, (M // 64, 8, 8, K), (0, 0, 0, 0), (1, 1), t).view(M, K), ref)
        ok = {t: v for t, v in res.items() if not isinstance(v, tuple)}
        best = min(ok, key=ok.get) if ok else None
        print(json.dumps({"pass": "dgrad", "M": M, "K": K, "N": N, "lib_ms": round(t_lib, 4),
                          "ws_ms": round(ok[best], 4) if best else None, "tile": best,
                          "bad": [t for t, v in res.items() if isinstance(v, tuple)],
                          "all": {"%d/%d/%d/%d" % t: round(v, 4) for t, v in sorted(ok.items(), key=lambda kv: kv[1])[:6]}}),
              flush=True)


if __name__ == "__main__":
    main()
