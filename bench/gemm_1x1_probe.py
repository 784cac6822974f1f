#!/usr/bin/env python
"""hipBLASLt (torch.mm) vs the mdtf conv kernels on ResNet-50's 1x1 (stride 1) convolutions as plain GEMMs:
fwd Y = X W, dgrad DX = DY W^T, at batch 256 (diagnostic)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench.conv_autotune import timeit  # noqa: E402
from mdtf.ops import conv as C  # noqa: E402

SHAPES = [(56, 64, 256), (56, 64, 64), (56, 256, 64), (56, 256, 128), (28, 128, 512), (28, 512, 128),
          (28, 512, 256), (14, 256, 1024), (14, 1024, 256), (14, 1024, 512), (7, 512, 2048), (7, 2048, 512)]


def main():
    dev = "cuda"
    print("| HxW | Cin | Cout | fwd mm ms | fwd mdtf ms (table) | dgrad mm ms | dgrad mdtf ms (table) | mem floor ms |")
    print("|---|---|---|---|---|---|---|---|")
    for h, ci, co in SHAPES:
        M = 256 * h * h
        x = torch.randn(M, ci, device=dev).bfloat16()
        w = (torch.randn(ci, co, device=dev) * 0.05).bfloat16()
        dy = torch.randn(M, co, device=dev).bfloat16()
        wt = w.t().contiguous()
        t_f = timeit(lambda: torch.mm(x, w), 10)
        t_d = timeit(lambda: torch.mm(dy, wt), 10)
        x4, w4, dy4 = x.view(256, h, h, ci), w.view(1, 1, ci, co), dy.view(256, h, h, co)
        pads = (0, 0, 0, 0)
        cf = C.choose("fwd", x4.shape, w4.shape, (1, 1), pads, (1, 1))
        cd = C.choose("dgrad", x4.shape, w4.shape, (1, 1), pads, (1, 1))
        st = torch.zeros(2, 1024, co, device=dev)
        tm_f = tm_d = float("nan")
        if cf[0] == "mdtf":
            tm_f = timeit(lambda: C.mdtf_fwd(x4, w4, (h, h), (1, 1), pads, (1, 1), cf[1], cf[2], (st[0], st[1]),
                                             cf[4], cf[5]), 10)
        if cd[0] == "mdtf":
            tm_d = timeit(lambda: C.mdtf_dgrad(dy4, w4, x4.shape, (1, 1), pads, (1, 1), cd[1], cd[2], cd[4], cd[5]), 10)
        floor = 2.0 * M * (ci + co) / 5.5e9
        print("| %d | %d | %d | %.3f | %.3f | %.3f | %.3f | %.3f |" % (h, ci, co, t_f, tm_f, t_d, tm_d, floor),
              flush=True)


if __name__ == "__main__":
    main()
