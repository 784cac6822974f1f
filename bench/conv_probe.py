#!/usr/bin/env python
"""Time every conv tile candidate for a few shapes, forward with and without the fused BN statistics
(diagnostic companion of bench/conv_autotune.py).  usage: conv_probe.py "N,H,W,C,K,CO,S" ..."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdtf.ops import conv as C  # noqa: E402
from bench.conv_autotune import V2_TILES, V3_TILES, timeit  # noqa: E402


def main():
    dev = "cuda"
    for spec in sys.argv[1:]:
        n, h, w, c, k, co, s = (int(v) for v in spec.split(","))
        p = k // 2
        pads = (p, p, p, p)
        oh, ow = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
        x = torch.randn(n, h, w, c, device=dev).bfloat16()
        wt = (torch.randn(k, k, c, co, device=dev) * 0.05).bfloat16()
        flops = 2.0 * n * oh * ow * co * k * k * c
        byts = 2.0 * (n * h * w * c + n * oh * ow * co)
        st = torch.zeros(2, 1024, co, device=dev)
        print("## fwd %s  (%.1f GFLOP, %.0f MB in+out)" % (spec, flops / 1e9, byts / 1e6))
        t = timeit(lambda: C.miopen_fwd(x, wt, (s, s), pads, (1, 1)), 10)
        print("miopen %.3f ms" % t)
        cands = [(bm, bn, 0, 1) for bm, bn in ((128, 128), (128, 64), (64, 64), (256, 64))]
        cands += [(bm, bn, sg, 2) for bm, bn, sg in V2_TILES] + [(bm, bn, sg, 3) for bm, bn, sg in V3_TILES]
        for bm, bn, sg, v in cands:
            try:
                t0 = timeit(lambda: C.mdtf_fwd(x, wt, (oh, ow), (s, s), pads, (1, 1), bm, bn, None, v, sg), 10)
                t1 = timeit(lambda: C.mdtf_fwd(x, wt, (oh, ow), (s, s), pads, (1, 1), bm, bn, (st[0], st[1]), v,
                                               sg), 10)
            except RuntimeError:
                continue
            print("v%d %3dx%3d s%d  %.3f ms  stats %.3f ms   %5.0f TF/s  %5.0f GB/s" % (
                v, bm, bn, sg, t0, t1, flops / t1 / 1e9, byts / t1 / 1e6))


if __name__ == "__main__":
    main()
