#!/usr/bin/env python
"""ResNet stem (7x7 s2, 3 -> 64 channels, batch 256, 224x224) on MIOpen vs the mdtf v1 kernel with the
input zero-padded to 8 channels (the mdtf kernels need Cin % 8 == 0).  Prints ms per forward and wgrad."""
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdtf.ops import conv as C  # noqa: E402


def timeit(fn, reps=10, warm=3):
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
    dev = "cuda"
    n = 256
    x3 = torch.randn(n, 224, 224, 3, device=dev).bfloat16()
    w3 = (torch.randn(7, 7, 3, 64, device=dev) * 0.05).bfloat16()
    x8 = torch.nn.functional.pad(x3, (0, 5))
    w8 = torch.nn.functional.pad(w3, (0, 0, 0, 5))
    xc = x3.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
    wc = w3.permute(3, 2, 0, 1).contiguous(memory_format=torch.channels_last)
    t_mi = timeit(lambda: torch.nn.functional.conv2d(xc, wc, stride=2, padding=3))
    print("MIOpen fwd (channels_last, 3 ch): %.3f ms" % t_mi, flush=True)
    t_pad = timeit(lambda: torch.nn.functional.pad(x3, (0, 5)))
    print("pad 3->8 channels: %.3f ms" % t_pad, flush=True)
    ref = torch.nn.functional.conv2d(xc.float(), wc.float(), stride=2, padding=3).permute(0, 2, 3, 1)
    for bm, bn in ((128, 64), (256, 64), (64, 64), (128, 128)):
        try:
            t = timeit(lambda: C.mdtf_fwd(x8, w8, (112, 112), (2, 2), (3, 3, 3, 3), (1, 1), bm, bn))
            y = C.mdtf_fwd(x8, w8, (112, 112), (2, 2), (3, 3, 3, 3), (1, 1), bm, bn)
            err = float((y.float() - ref).norm() / ref.norm())
            print("mdtf v1 fwd %dx%d: %.3f ms (err %.1e)" % (bm, bn, t, err), flush=True)
        except RuntimeError as e:
            print("mdtf v1 fwd %dx%d: %s" % (bm, bn, e), flush=True)
    dy = torch.randn(n, 112, 112, 64, device=dev).bfloat16()
    dyc = dy.permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
    t_mw = timeit(lambda: torch.ops.aten.convolution_backward(dyc, xc, wc, None, (2, 2), (3, 3), (1, 1), False, (0, 0),
                                                              1, (False, False, True)))
    print("MIOpen wgrad: %.3f ms" % t_mw, flush=True)
    for bm, bn, sp in ((64, 64, 0), (128, 64, 0), (64, 64, 16), (128, 64, 32)):
        for ver in (1,):
            try:
                t = timeit(lambda: C.mdtf_wgrad(x8, dy, (7, 7, 8, 64), (2, 2), (3, 3, 3, 3), (1, 1), bm, bn, sp,
                                                ver=ver))
                print("mdtf v%d wgrad %dx%d split %d: %.3f ms" % (ver, bm, bn, sp, t), flush=True)
            except RuntimeError as e:
                print("mdtf wgrad %dx%d: %s" % (bm, bn, e), flush=True)


if __name__ == "__main__":
    main()
