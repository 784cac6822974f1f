#!/usr/bin/env python
"""Weight-gradient GEMM micro-benchmark: dW[K][N] += X^T[K][M] dY[M][N] (fp32 accumulate).

Compares hipBLASLt (torch.addmm with out_dtype=float32 into the fp32 slot) with the
mdtf implicit-GEMM wgrad kernel run as a 1x1 convolution (v2: LDS-DMA + transposed
LDS reads, split-K fp32 atomics) at the BERT-base / ResNet FC shapes.
"""
import statistics
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdtf.ops import conv as C  # noqa: E402


def timeit(fn, reps=20, warm=5):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


def main():
    dev = torch.device("cuda")
    shapes = [(8192, 768, 768), (8192, 768, 3072), (8192, 3072, 768), (8192, 768, 2304), (1280, 768, 768)]
    print("| M | K | N | hipBLASLt ms | TF/s | mdtf best ms (tile) | TF/s |")
    print("|---|---|---|---|---|---|---|")
    for M, K, N in shapes:
        x = torch.randn(M, K, device=dev).bfloat16()
        dy = torch.randn(M, N, device=dev).bfloat16()
        out = torch.zeros(K, N, device=dev)
        fl = 2.0 * M * K * N
        t_lib = timeit(lambda: torch.addmm(out, x.t(), dy, out_dtype=torch.float32, out=out))
        xt = x.t()
        t_b16 = timeit(lambda: out.add_(torch.mm(xt, dy)))       # bf16-output GEMM + fp32 accumulate pass
        t_b16only = timeit(lambda: torch.mm(xt, dy))
        best = None
        x4 = x.view(M, 1, 1, K)
        dy4 = dy.view(M, 1, 1, N)
        for bm, bn, st, v in ((128, 128, 2, 2), (128, 128, 3, 2), (128, 128, 4, 2), (128, 128, 5, 2), (64, 128, 2, 2),
                              (64, 128, 4, 2), (64, 128, 6, 2), (128, 64, 2, 2), (64, 64, 3, 2),
                              (256, 256, 2, 3), (256, 128, 2, 3), (256, 128, 3, 3), (128, 256, 2, 3),
                              (128, 256, 3, 3), (128, 128, 3, 3), (128, 128, 4, 3), (128, 128, 5, 3)):
            for sp in (0, 1, 2, 3, 4, 8, 16):
                try:
                    t = timeit(lambda: C.mdtf_wgrad(x4, dy4, (1, 1, K, N), (1, 1), (0, 0, 0, 0), (1, 1), bm, bn, sp,
                                                    out=out, ver=v, stages=st))
                except RuntimeError:
                    continue
                if best is None or t < best[0]:
                    best = (t, bm, bn, st, sp, v)
        # numerics spot check
        out.zero_()
        C.mdtf_wgrad(x4, dy4, (1, 1, K, N), (1, 1), (0, 0, 0, 0), (1, 1), best[1], best[2], best[4], out=out,
                     ver=best[5], stages=best[3])
        ref = (x.t().float() @ dy.float())
        err = float((out.view(K, N) - ref).norm() / ref.norm())
        print("| %d | %d | %d | %.4f | %.0f | %.4f (%d,%d,s%d,k%d,v%d) | %.0f | bf16-out %.4f (+add %.4f) | err %.1e" % (
            M, K, N, t_lib, fl / t_lib / 1e9, best[0], best[1], best[2], best[3], best[4], best[5], fl / best[0] / 1e9,
            t_b16only, t_b16, err), flush=True)


if __name__ == "__main__":
    main()
