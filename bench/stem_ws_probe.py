#!/usr/bin/env python
"""ResNet stem forward (7x7/2, 3 -> 64, batch 256, 224x224, BN statistics fused): MIOpen (+ the separate
BN reduction it needs) vs the hand-written stem (repack + weight-stationary GEMM) for several tiles."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdtf.ops import conv as C  # noqa: E402


def timeit(fn, reps=20, warm=3):
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
    x = torch.randn(256, 224, 224, 3, device=dev).bfloat16()
    w = (torch.randn(7, 7, 3, 64, device=dev) * 0.05).bfloat16()
    pads = (3, 3, 3, 3)
    t_lib = timeit(lambda: C.miopen_fwd(x, w, (2, 2), pads, (1, 1)))
    sbuf = torch.zeros(2, 64, 64, device=dev)
    res = {"miopen_fwd_ms": round(t_lib, 4)}
    for tile in [(4, 8, 1, 4), (2, 8, 1, 4), (4, 4, 1, 4), (2, 4, 1, 4)]:
        res["stem_%d%d%d%d_ms" % tile] = round(timeit(lambda: C.stem_fwd(x, w, (112, 112), (2, 2), pads,
                                                                          (sbuf[0], sbuf[1]), tile)), 4)
    res["stem_rows_ms"] = round(timeit(lambda: C.stem_fwd(x, w, (112, 112), (2, 2), pads, (sbuf[0], sbuf[1]))), 4)
    xa = torch.empty(256, 230, 230, 4, device=dev, dtype=torch.bfloat16)
    from mdtf.ops import _native as N
    res["pack_ms"] = round(timeit(lambda: N.fn("mdtf_stem_pack4")(N.ptr(x), N.ptr(xa), 256, 224, 224, 3, 3, 3, 230,
                                                                   230, None, None, 0, 0, 0, 0,
                                                                   N.stream_ptr())), 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
