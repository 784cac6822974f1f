"""Graph-timed fan-out data gradient of a ResNet-50 projection block input (stages 2 and 3, batch 256): the fused
one-pass kernel (mdtf_conv_ws_dual, BN-backward statistics epilogue) vs the two data gradients the table would run
(the strided projection's, written; then conv1's, accumulating with the statistics), alternating in one process.
One JSON line per round and a median summary."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from bench.gemm_pp_probe import gtime  # noqa: E402
from mdtf.ops import conv as C  # noqa: E402

SHAPES = {"stage2": (56, 256, 128, 512), "stage3": (28, 512, 256, 1024)}


def _dgrad(dy, w, x_shape, stride, out=None, accumulate=False, bn_stats=None):
    cd = C.choose("dgrad", x_shape, tuple(w.shape), stride, (0, 0, 0, 0), (1, 1))
    if cd[0] == "ws":
        return C.ws_dgrad(dy, w, x_shape, (0, 0, 0, 0), (1, 1), (2,) + tuple(cd[1][1:]) if bn_stats else cd[1],
                          out=out, accumulate=accumulate, bn_stats=bn_stats)
    if cd[0] == "pp":
        return C.pp_dgrad(dy, w, x_shape, (0, 0, 0, 0), (1, 1), cd[1], out=out, accumulate=accumulate,
                          bn_stats=bn_stats)
    return C.mdtf_dgrad(dy, w, x_shape, stride, (0, 0, 0, 0), (1, 1), cd[1], cd[2], cd[4], cd[5], out=out,
                        accumulate=accumulate, bn_stats=bn_stats)


def main():
    n = int(os.environ.get("B", "256"))
    dev = "cuda"
    res = {}
    for name, (h, c, c1, c2) in SHAPES.items():
        xs = (n, h, h, c)
        dy1 = torch.randn(n, h, h, c1, device=dev).bfloat16()
        dy2 = torch.randn(n, h // 2, h // 2, c2, device=dev).bfloat16()
        w1 = (torch.randn(1, 1, c, c1, device=dev) / c ** 0.5).bfloat16()
        w2 = (torch.randn(1, 1, c, c2, device=dev) / c ** 0.5).bfloat16()
        bx = torch.randn(xs, device=dev).bfloat16()
        mask = torch.randint(0, 256, (n * h * h * c // 8,), device=dev, dtype=torch.uint8)
        sb = torch.zeros(2, C.STAT_SLOTS, c, device=dev)
        bst = (bx, mask, sb[0], sb[1], C.STAT_SLOTS)
        out = torch.empty(xs, device=dev, dtype=torch.bfloat16)

        def fused():
            C.ws_dual(dy1, w1, (dy2, w2, (2, 2)), xs, tile=(2, 8, 1), bn_stats=bst)

        def fused241():
            C.ws_dual(dy1, w1, (dy2, w2, (2, 2)), xs, tile=(2, 4, 1), bn_stats=bst)

        def split():
            _dgrad(dy2, w2, xs, (2, 2), out=out)
            _dgrad(dy1, w1, xs, (1, 1), out=out, accumulate=True, bn_stats=bst)

        res[name] = {"fused": [], "fused241": [], "split": []}
        for rnd in range(5):
            for arm, fn in (("fused", fused), ("fused241", fused241), ("split", split)):
                t = gtime(fn) * 1000.0
                res[name][arm].append(t)
                print(json.dumps({"shape": name, "round": rnd, "arm": arm, "us": round(t, 2)}), flush=True)
    print(json.dumps({"summary": {k: {a: round(statistics.median(v), 2) for a, v in d.items()} for k, d in res.items()},
                      "B": n}), flush=True)


if __name__ == "__main__":
    main()
