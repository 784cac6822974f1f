#!/usr/bin/env python
"""Stem forward variants for counter passes and timing (batch 256, 224x224x3 -> 112x112x64, 7x7/2):
row-staged kernel with / without the fused BN statistics, and the streamed weight-stationary kernel."""
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
    pads = (3, 3, 3, 3)
    sbuf = torch.zeros(2, 64, 64, device=dev)
    runs = {"rows_stats": lambda: C.stem_fwd(x, w, (112, 112), (2, 2), pads, (sbuf[0], sbuf[1])),
            "rows_nostats": lambda: C.stem_fwd(x, w, (112, 112), (2, 2), pads, None),
            "ws_stats": lambda: C.stem_fwd(x, w, (112, 112), (2, 2), pads, (sbuf[0], sbuf[1]), C.STEM_TILE)}
    res = {k: round(timeit(f, reps=int(os.environ.get("REPS", "10")), warm=2), 4) for k, f in runs.items()}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
