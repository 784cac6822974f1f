#!/usr/bin/env python
"""Dense forward on the hand-written MFMA kernel (ops/gemm.py hand_fwd: fd v2 MODE 3, W read in place,
bias + activation epilogue, q|k|v segments) vs hipBLASLt (addmm with the bias epilogue, + the mdtf activation
kernel for GELU) on the BERT-base shapes, every candidate tile, timed inside captured graphs; prints one JSON
line per shape."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdtf.ops import gemm as G  # noqa: E402
from mdtf.ops import tunable  # noqa: E402

# (M, K, segment width, segments, act): BERT-base at batch 64 x seq 128 (qkv, attention out, FFN in/out)
SHAPES = [(8192, 768, 768, 3, 0), (8192, 768, 768, 1, 0), (8192, 768, 3072, 1, 2), (8192, 3072, 768, 1, 0),
          (1280, 768, 768, 1, 0)]
TILES = [(128, 128, 2, 2), (128, 128, 3, 2), (128, 128, 4, 2), (128, 64, 3, 2), (64, 128, 3, 2), (256, 128, 2, 3),
         (256, 128, 3, 3), (256, 256, 2, 3), (128, 256, 2, 3), (128, 256, 3, 3), (256, 64, 3, 3), (256, 64, 4, 3)]


def timeit(fn, reps=20):
    """Kernel time per call inside a captured graph (as in the training step: no host launch cost, which
    inflates an eagerly timed hipBLASLt call by up to 50 %)."""
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


def main():
    dev = torch.device("cuda")
    tunable.ensure(dev)
    for M, K, nw, nseg, act in SHAPES:
        x = torch.randn(M, K, device=dev).bfloat16()
        ws = [(torch.randn(K, nw, device=dev) * 0.03).bfloat16() for _ in range(nseg)]
        b = (torch.randn(nw * nseg, device=dev) * 0.1).bfloat16()

        def lib():
            w = ws[0] if nseg == 1 else torch.cat(ws, 1)
            pre = torch.addmm(b, x, w)
            return G._act_fwd(pre, act) if act else pre
        t_lib = timeit(lib)
        res = {}
        for tile in TILES:
            if nw % tile[1]:
                continue
            if G.hand_fwd(x, ws, b, act, tile=tile) is None:
                continue
            res[tile] = timeit(lambda: G.hand_fwd(x, ws, b, act, tile=tile))
        best = min(res, key=res.get)
        y, _ = G.hand_fwd(x, ws, b, act, tile=best)
        ref = lib().float()
        err = ((y.float() - ref).norm() / ref.norm()).item()
        fl = 2.0 * M * K * nw * nseg
        print(json.dumps({"M": M, "K": K, "N": nw, "seg": nseg, "act": act, "lib_ms": round(t_lib, 4),
                          "mdtf_ms": round(res[best], 4), "tile": best, "lib_TFs": round(fl / t_lib / 1e9),
                          "mdtf_TFs": round(fl / res[best] / 1e9), "rel_err_vs_lib": round(err, 5),
                          "all": {"%d/%d/%d/%d" % t: round(v, 4) for t, v in sorted(res.items(), key=lambda kv: kv[1])}}),
              flush=True)


if __name__ == "__main__":
    main()
