#!/usr/bin/env python
"""Weight-gradient kernel probe: steady-state vs split-K cost of conv_wgrad_v2.

dW[K][N] += X^T[K][M] dY[M][N] run as a 1x1 convolution, per tile / split count, with
split-K partials added by fp32 atomics or written to a slab and reduced.  A large-output
shape (no split needed) gives the kernel's steady-state MFMA rate; the BERT / ResNet
shapes show what split-K costs on top of it.

    python bench/wgrad_probe.py [--quick]
"""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdtf.ops import conv as C  # noqa: E402


def timeit(fn, reps=15, warm=3):
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


def one(argv):
    """--one M K N bm bn stages ver splits slab: 20 launches of one config (for rocprofv3 --pmc)."""
    M, K, N, bm, bn, st, v, sp, slab = [int(a) for a in argv]
    x = torch.randn(M, K, device="cuda").bfloat16().view(M, 1, 1, K)
    dy = torch.randn(M, N, device="cuda").bfloat16().view(M, 1, 1, N)
    out = torch.zeros(K, N, device="cuda")
    C.WGRAD_SLAB = bool(slab)
    for _ in range(20):
        C.mdtf_wgrad(x, dy, (1, 1, K, N), (1, 1), (0, 0, 0, 0), (1, 1), bm, bn, sp, out=out, ver=v, stages=st)
    torch.cuda.synchronize()
    print("ok")


def main():
    if "--one" in sys.argv:
        return one(sys.argv[sys.argv.index("--one") + 1:])
    quick = "--quick" in sys.argv
    dev = torch.device("cuda")
    shapes = [(8192, 4096, 4096), (8192, 768, 3072), (8192, 3072, 768), (50176, 256, 256), (12544, 512, 2048)]
    tiles = [(64, 128, 2, 2), (128, 128, 2, 2), (128, 128, 3, 2), (256, 256, 2, 3), (256, 128, 2, 3),
             (128, 256, 2, 3), (128, 128, 2, 3)]
    split_opts = (1, 2, 4, 8, 16, 32) if not quick else (1, 4, 16)
    print("| M | K | N | tile | splits | atomics ms | TF/s | slab ms | TF/s |")
    print("|---|---|---|---|---|---|---|---|---|")
    for M, K, N in shapes:
        x = torch.randn(M, K, device=dev).bfloat16().view(M, 1, 1, K)
        dy = torch.randn(M, N, device=dev).bfloat16().view(M, 1, 1, N)
        out = torch.zeros(K, N, device=dev)
        fl = 2.0 * M * K * N
        best = None
        for bm, bn, st, v in tiles:
            for sp in split_opts:
                row = []
                for slab in (False, True):
                    if slab and sp < 2:
                        row.append(None)
                        continue
                    C.WGRAD_SLAB = slab
                    try:
                        t = timeit(lambda: C.mdtf_wgrad(x, dy, (1, 1, K, N), (1, 1), (0, 0, 0, 0), (1, 1), bm, bn, sp,
                                                        out=out, ver=v, stages=st))
                    except RuntimeError:
                        t = None
                    row.append(t)
                    if t is not None and (best is None or t < best[0]):
                        best = (t, bm, bn, st, v, sp, slab)
                if row[0] is None and row[1] is None:
                    continue
                f = lambda t: ("%.4f | %.0f" % (t, fl / t / 1e9)) if t else "- | -"
                print("| %d | %d | %d | %dx%d s%d v%d | %d | %s | %s |" % (M, K, N, bm, bn, st, v, sp, f(row[0]),
                                                                         f(row[1])), flush=True)
        print("best %dx%dx%d: %.4f ms %.0f TF/s %s" % (M, K, N, best[0], fl / best[0] / 1e9, best[1:]), flush=True)


if __name__ == "__main__":
    main()
