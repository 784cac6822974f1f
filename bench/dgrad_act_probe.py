#!/usr/bin/env python
"""FFN second-layer data gradient with the GELU backward fused into the epilogue (ops/gemm.py hand_dgrad_act)
vs hipBLASLt + the separate activation-backward kernel, graph-timed, every candidate tile (BERT-base shapes)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdtf.ops import gemm as G  # noqa: E402
from mdtf.ops import tunable  # noqa: E402
from bench.dense_fwd_probe import TILES, timeit  # noqa: E402

SHAPES = [(8192, 3072, 768), (1280, 3072, 768)]     # (M, K = intermediate, N = hidden)


def main():
    dev = torch.device("cuda")
    tunable.ensure(dev)
    for M, K, Nn in SHAPES:
        dy = torch.randn(M, Nn, device=dev).bfloat16()
        w = (torch.randn(K, Nn, device=dev) * 0.03).bfloat16()
        pre = torch.randn(M, K, device=dev).bfloat16()
        t_lib = timeit(lambda: G._act_bwd(torch.mm(dy, w.t()), pre, 2))
        t_mm = timeit(lambda: torch.mm(dy, w.t()))
        ref = G._act_bwd(torch.mm(dy, w.t()), pre, 2).float()
        res = {}
        for t in TILES:
            dx = G.hand_dgrad_act(dy, w, pre, 2, tile=t)
            if dx is None:
                continue
            err = ((dx.float() - ref).norm() / ref.norm()).item()
            if err > 2e-2:
                res[t] = -err
                continue
            res[t] = timeit(lambda: G.hand_dgrad_act(dy, w, pre, 2, tile=t))
        ok = {t: v for t, v in res.items() if v > 0}
        best = min(ok, key=ok.get)
        print(json.dumps({"M": M, "K": K, "N": Nn, "lib_mm_plus_act_ms": round(t_lib, 4), "lib_mm_ms": round(t_mm, 4),
                          "fused_ms": round(ok[best], 4), "tile": best,
                          "bad": ["%d/%d/%d/%d" % t for t, v in res.items() if v <= 0],
                          "all": {"%d/%d/%d/%d" % t: round(v, 4) for t, v in sorted(ok.items(), key=lambda kv: kv[1])[:6]}}),
              flush=True)


if __name__ == "__main__":
    main()
