#!/usr/bin/env python
"""Stem weight gradient (csrc/stem_wgrad.hip) at ResNet-50's shape (batch 256, x4 230x230, dy 112x112x64) for
several grid sizes (blocks of 8 waves splitting the 32-pixel k-steps)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdtf.ops import conv as C  # noqa: E402
from stem_ws_probe import timeit  # noqa: E402


def main():
    dev = "cuda"
    x = torch.randn(256, 224, 224, 3, device=dev).bfloat16()
    w = (torch.randn(7, 7, 3, 64, device=dev) * 0.05).bfloat16()
    keep = []
    C.stem_fwd(x, w, (112, 112), (2, 2), (3, 3, 3, 3), None, keep_x4=keep)
    dy = torch.randn(256, 112, 112, 64, device=dev).bfloat16()
    dw = torch.zeros(7, 7, 3, 64, device=dev)
    res = {}
    for blocks in (256, 512, 768, 1024, 2048):
        res["blocks_%d_ms" % blocks] = round(timeit(lambda: C.stem_wgrad(keep[0], dy, w.shape, (2, 2), dw, blocks),
                                                    reps=10, warm=2), 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
