"""Graph-timed ResNet-50 stage-1 3x3 convolution (batch 256, 56 x 56, 64 -> 64 channels): the row-staged kernel
(csrc/conv_rows.hip) vs the streamed weight-stationary kernel (csrc/conv_ws.hip) it replaces, forward with the
BN-statistics epilogue and data gradient with the BN-backward statistics, alternating in one process.  One JSON
line per round and a median summary."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from bench.gemm_pp_probe import gtime  # noqa: E402
from mdtf.ops import conv as C  # noqa: E402


def main():
    n, h, w, c = int(os.environ.get("B", "256")), 56, 56, 64
    dev = "cuda"
    pads = (1, 1, 1, 1)
    x = torch.randn(n, h, w, c, device=dev).bfloat16()
    wt = (torch.randn(3, 3, c, c, device=dev) / 24.0).bfloat16()
    wtt = C.transpose_filter(wt)
    dy = torch.randn(n, h, w, c, device=dev).bfloat16()
    bx = torch.randn(n, h, w, c, device=dev).bfloat16()
    mask = torch.randint(0, 256, (n * h * w * c // 8,), device=dev, dtype=torch.uint8)
    sb = torch.zeros(2, 8, c, device=dev)
    y = torch.empty_like(x)
    dx = torch.empty_like(x)
    fwd = lambda: C.ws_fwd(x, wtt, 3, 3, (h, w), (1, 1), pads, (1, 1), (4, 8, 1, 3), (sb[0], sb[1]), out=y)  # noqa
    bwd = lambda: C.ws_dgrad(dy, wt, (n, h, w, c), pads, (1, 1), (2, 8, 1, 3), out=dx,  # noqa
                             bn_stats=(bx, mask, sb[0], sb[1], 8))
    fl = 2.0 * n * h * w * c * c * 9
    res = {0: {"fwd": [], "bwd": []}, 1: {"fwd": [], "bwd": []}}
    for rnd in range(5):
        for rows in (0, 1):
            C.CONV_ROWS = bool(rows)
            tf = gtime(fwd) * 1000.0
            tb = gtime(bwd) * 1000.0
            res[rows]["fwd"].append(tf)
            res[rows]["bwd"].append(tb)
            print(json.dumps({"round": rnd, "rows": rows, "fwd_us": round(tf, 2), "bwd_us": round(tb, 2)}), flush=True)
    summ = {}
    for rows in (0, 1):
        f, b = statistics.median(res[rows]["fwd"]), statistics.median(res[rows]["bwd"])
        summ["rows%d" % rows] = {"fwd_us": round(f, 2), "bwd_us": round(b, 2), "fwd_TFs": round(fl / f / 1e6, 1),
                                 "bwd_TFs": round(fl / b / 1e6, 1)}
    print(json.dumps({"summary": summ, "B": n}), flush=True)


if __name__ == "__main__":
    main()
