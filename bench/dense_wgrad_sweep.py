#!/usr/bin/env python
"""Dense weight-gradient tile sweep, timed inside captured graphs (kernel time only, as in the training step):
dW[K][N] (fp32) += X[M][K]^T dY[M][N] on the hand-written v2 wgrad kernel over every instantiated tile x split
count x (slab reduction | fp32 atomics), vs the current ops/gemm.py choice and hipBLASLt's fp32-output GEMM.
Prints one JSON line per BERT-base shape."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdtf.ops import _native as N  # noqa: E402
from mdtf.ops import conv as C  # noqa: E402
from mdtf.ops import gemm as G  # noqa: E402

SHAPES = [(8192, 768, 768), (8192, 768, 3072), (8192, 3072, 768), (1280, 768, 768)]
# (bm, bn, stages, 8 waves)
TILES = [(128, 128, 2, 0), (128, 128, 3, 0), (128, 64, 2, 0), (128, 64, 3, 0), (64, 128, 2, 0), (64, 128, 3, 0),
         (64, 64, 2, 0), (64, 64, 3, 0), (64, 64, 4, 0), (256, 256, 2, 1), (256, 128, 2, 1), (256, 128, 3, 1),
         (128, 256, 2, 1), (128, 256, 3, 1), (128, 128, 2, 1), (128, 128, 3, 1), (128, 128, 4, 1), (128, 128, 5, 1),
         (128, 128, 4, 0), (128, 128, 5, 0), (64, 128, 4, 0), (64, 128, 6, 0)]
SPLITS = [0, 1, 2, 4, 8, 16]


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


def launch(x, d, out, bm, bn, st, w8, splits, slab_on, dbias=None):
    M, K = x.shape
    Nn = d.shape[1]
    slab, cap = (C.wgrad_slab(M, K, Nn, bm, bn, 3 if w8 else 2, splits, x.device, dense=True) if slab_on
                 else (None, 0))
    rc = N.fn("mdtf_gemm_wgrad")(N.ptr(x), N.ptr(d), N.ptr(out), M, K, Nn, d.stride(0), out.stride(0),
                                 bm + 10000 * w8, bn, st, splits, N.ptr(slab), cap, N.ptr(dbias), N.stream_ptr())
    if rc != 0:
        raise RuntimeError("rc %d" % rc)


def main():
    dev = torch.device("cuda")
    for M, K, Nn in SHAPES:
        x = torch.randn(M, K, device=dev).bfloat16()
        d = torch.randn(M, Nn, device=dev).bfloat16()
        out = torch.zeros(K, Nn, device=dev)
        ref = x.float().t() @ d.float()
        t_cur = gtime(lambda: G.wgrad_into(out, x, d))
        t_lib = gtime(lambda: G._accum_mm(out, x.t(), d))
        res = {}
        for bm, bn, st, w8 in TILES:
            for sp in SPLITS:
                for slab_on in (True, False):
                    key = (bm, bn, st, w8, sp, int(slab_on))
                    try:
                        out.zero_()
                        launch(x, d, out, bm, bn, st, w8, sp, slab_on)
                        torch.cuda.synchronize()
                    except RuntimeError:
                        continue
                    err = ((out - ref).norm() / ref.norm()).item()
                    if err > 1e-2:
                        res[key] = None
                        continue
                    res[key] = gtime(lambda: launch(x, d, out, bm, bn, st, w8, sp, slab_on))
        ok = {k: v for k, v in res.items() if v is not None}
        best = sorted(ok.items(), key=lambda kv: kv[1])[:8]
        print(json.dumps({"M": M, "K": K, "N": Nn, "current_ms": round(t_cur, 4), "hipblaslt_fp32_ms": round(t_lib, 4),
                          "best": [[list(k), round(v, 4)] for k, v in best],
                          "bad": [list(k) for k, v in res.items() if v is None]}), flush=True)


if __name__ == "__main__":
    main()
