#!/usr/bin/env python
"""Weight-stationary conv kernel (csrc/conv_ws.hip) vs the table's current choice on the ResNet-50
shapes it takes (batch 256): forward (with the BN-statistics epilogue) and stride-1 dgrad.
Prints one line per (pass, shape, tile) with ms and the HBM-floor ratio."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdtf.ops import conv as C  # noqa: E402

SHAPES = [  # (H, Cin, k, Cout, stride)  as they appear in ResNet-50 (input side)
    (56, 64, 1, 256, 1), (56, 64, 1, 64, 1), (56, 256, 1, 64, 1), (56, 256, 1, 128, 1), (56, 256, 1, 512, 2),
    (56, 64, 3, 64, 1), (28, 128, 1, 512, 1), (28, 512, 1, 128, 1), (28, 128, 3, 128, 1), (14, 256, 1, 1024, 1),
    (14, 1024, 1, 256, 1),
]
TILES = [(4, 8, 1, 4), (4, 8, 2, 4), (4, 8, 4, 4), (4, 8, 1, 6), (4, 8, 2, 6), (4, 8, 4, 6), (2, 8, 1, 4),
         (2, 8, 2, 4), (2, 8, 1, 8), (2, 8, 2, 8), (2, 8, 4, 8), (4, 4, 1, 4), (4, 4, 1, 6), (2, 4, 1, 8)]


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--out", default=None)
    ap.add_argument("--isolate", action="store_true", help="also time the first tile without stores / loads")
    ap.add_argument("--tiles", default=None, help="tp,nw,cg,d;... subset")
    ap.add_argument("--shapes", default=None, help="indices into SHAPES, comma-separated")
    a = ap.parse_args()
    dev = torch.device("cuda")
    global TILES
    if a.tiles:
        TILES = [tuple(int(v) for v in t.split(",")) for t in a.tiles.split(";")]
    recs = []
    shapes = [SHAPES[int(i)] for i in a.shapes.split(",")] if a.shapes else SHAPES
    for (h, c, k, co, s) in shapes:
        p = k // 2
        oh = (h + 2 * p - k) // s + 1
        x = torch.randn(a.batch, h, h, c, device=dev).bfloat16()
        w = (torch.randn(k, k, c, co, device=dev) / (k * k * c) ** 0.5).bfloat16()
        wt = C.transpose_filter(w)
        pads = (p, p, p, p)
        dy = torch.randn(a.batch, oh, oh, co, device=dev).bfloat16()
        floor_f = (x.numel() + dy.numel()) * 2 / 5.5e12 * 1e3        # ms at 5.5 TB/s
        for pass_ in ("fwd", "dgrad"):
            if pass_ == "dgrad" and s != 1:
                continue
            ch = C.choose(pass_, x.shape, w.shape, (s, s), pads, (1, 1))
            sbuf = torch.zeros(2, 64, co if pass_ == "fwd" else c, device=dev)
            if ch[0] == "ws":
                if pass_ == "fwd":
                    base = lambda: C.ws_fwd(x, wt, k, k, (oh, oh), (s, s), pads, (1, 1), ch[1],  # noqa: E731
                                            (sbuf[0], sbuf[1]))
                else:
                    base = lambda: C.ws_dgrad(dy, w, x.shape, pads, (1, 1), ch[1])  # noqa: E731
            elif pass_ == "fwd":
                if ch[0] == "mdtf":
                    base = lambda: C.mdtf_fwd(x, w, (oh, oh), (s, s), pads, (1, 1), ch[1], ch[2],  # noqa: E731
                                              (sbuf[0], sbuf[1]), ch[4], ch[5])
                else:
                    base = lambda: C.miopen_fwd(x, w, (s, s), pads, (1, 1))  # noqa: E731
            else:
                base = lambda: C.mdtf_dgrad(dy, w, x.shape, (s, s), pads, (1, 1), ch[1], ch[2], ch[4], ch[5])  # noqa
            tb = timeit(base)
            best = None
            for tile in TILES:
                ncol = co if pass_ == "fwd" else c
                if ncol % (64 * tile[2]) or not C.ws_ok(pass_, c, co, (s, s), k, k):
                    continue
                if 64 * tile[2] * k * k * (c if pass_ == "fwd" else co) * 2 > 160 * 1024:
                    continue
                if pass_ == "fwd":
                    fn = lambda: C.ws_fwd(x, wt, k, k, (oh, oh), (s, s), pads, (1, 1), tile, (sbuf[0], sbuf[1]))  # noqa
                else:
                    fn = lambda: C.ws_dgrad(dy, w, x.shape, pads, (1, 1), tile)  # noqa: E731
                try:
                    t = timeit(fn)
                except RuntimeError as e:
                    print("skip", pass_, h, c, k, co, s, tile, e, flush=True)
                    continue
                extra = {}
                if a.isolate and best is None:
                    import ctypes
                    from mdtf.ops import _native as NN
                    for mode, name in ((1, "no_store_ms"), (2, "no_load_ms"), (3, "compute_only_ms"),
                                       (6, "store_only_ms"), (5, "load_only_ms")):
                        NN.lib().mdtf_conv_ws_debug(ctypes.c_int(mode))
                        extra[name] = round(timeit(fn), 4)
                    NN.lib().mdtf_conv_ws_debug(ctypes.c_int(0))
                rec = {"pass": pass_, "shape": [h, c, k, co, s], "tile": tile, "ws_ms": round(t, 4),
                       "cur_ms": round(tb, 4), "cur": list(ch), "floor_ms": round(floor_f, 4), **extra}
                print(json.dumps(rec), flush=True)
                recs.append(rec)
                if best is None or t < best[0]:
                    best = (t, tile)
            if best:
                print("BEST %s %s: ws %.4f (%s) vs current %.4f ms (floor %.4f)" % (
                    pass_, (h, c, k, co, s), best[0], best[1], tb, floor_f), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(recs, f, indent=1)


if __name__ == "__main__":
    main()
