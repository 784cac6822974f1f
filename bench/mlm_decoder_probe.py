"""Graph-timed BERT-base tied MLM decoder products (1280 masked rows x 768 x 30522) on hipBLASLt, as the step runs
them and in the layouts a padded vocabulary (30720 = 240 x 128 rows of the bf16 weight shadow) would allow:

  fwd     logits = h W^T                 [1280, 30522]   (step: MT256x224 tile)
  dx      dh = dlogits W                  [1280, 768], K = 30522: 80 output tiles, no split-K in the step
  dw      gW += dlogits^T h  (fp32 slot)  [30522, 768], K = 1280

Variants of dx: the transposed problem (dh^T = W^T dlogits^T), fp32 output, and split-K as a batched product over
S vocabulary chunks of the padded layout (fp32 partials summed).  One JSON line per (variant, round), then medians.
"""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from bench.gemm_pp_probe import gtime  # noqa: E402


def main():
    dev = "cuda"
    M, H, V, VP = 1280, 768, 30522, 30720
    torch.manual_seed(0)
    h = (torch.rand(M, H, device=dev) * 2 - 1).bfloat16()
    W = (torch.rand(V, H, device=dev) * 0.1 - 0.05).bfloat16()
    Wp = torch.zeros(VP, H, device=dev, dtype=torch.bfloat16)
    Wp[:V] = W
    d = (torch.rand(M, V, device=dev) * 2e-3 - 1e-3).bfloat16()
    dp = torch.zeros(M, VP, device=dev, dtype=torch.bfloat16)
    dp[:, :V] = d
    g = torch.zeros(V, H, device=dev)
    gp = torch.zeros(VP, H, device=dev)
    ref = (d.float() @ W.float())

    def split(S):
        def f():
            part = torch.bmm(dp.view(M, S, VP // S).transpose(0, 1), Wp.view(S, VP // S, H), out_dtype=torch.float32)
            return part.sum(0).to(torch.bfloat16)
        return f

    arms = {
        "fwd": lambda: torch.mm(h, W.t()),
        "fwd_pad": lambda: torch.mm(h, Wp.t()),
        "dx": lambda: torch.mm(d, W),
        "dx_pad": lambda: torch.mm(dp, Wp),
        "dx_T": lambda: torch.mm(W.t(), d.t()),
        "dx_f32": lambda: torch.mm(d, W, out_dtype=torch.float32),
        "dx_split4": split(4),
        "dx_split8": split(8),
        "dx_split16": split(16),
        "dw": lambda: torch.addmm(g, d.t(), h, out_dtype=torch.float32, out=g),
        "dw_pad": lambda: torch.addmm(gp, dp.t(), h, out_dtype=torch.float32, out=gp),
    }
    for S in (4, 8, 16):
        err = (split(S)().float() - ref).abs().max().item() / ref.abs().max().item()
        print(json.dumps({"check": "dx_split%d" % S, "max_rel_err": err}), flush=True)
    res = {a: [] for a in arms}
    for rnd in range(3):
        for arm, fn in arms.items():
            t = gtime(fn) * 1000.0
            res[arm].append(t)
            print(json.dumps({"arm": arm, "round": rnd, "us": round(t, 2)}), flush=True)
    print(json.dumps({"summary": {a: round(statistics.median(v), 2) for a, v in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
