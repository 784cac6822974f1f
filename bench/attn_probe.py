"""Graph-timed S = 128 fused attention at BERT-base shapes (batch 64, 12 heads, head dim 64, dropout 0.1):
per-item kernels (attn_fwd_kernel / attn_bwd_v2) vs the persistent forms (attn_fwd_pp / attn_bwd_pp), alternating
in one process (cdna_hip_programming.md §5.4 rule 24).  One JSON line per round and a median summary."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from bench.gemm_pp_probe import gtime  # noqa: E402
from mdtf.ops import _native as N  # noqa: E402
from mdtf.ops import transformer as T  # noqa: E402


def main():
    B, S, nh, dh, p = int(os.environ.get("B", "64")), 128, 12, 64, 0.1
    H = nh * dh
    dev = "cuda"
    qkv = (torch.randn(B * S, 3 * H, device=dev) * 0.5).bfloat16()
    mask = (torch.rand(B, S, device=dev) < 0.15).float() * -10000.0
    out = torch.empty(B * S, H, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * nh, S, device=dev)
    dout = torch.randn(B * S, H, device=dev).bfloat16()
    dqkv = torch.empty_like(qkv)
    scale = dh ** -0.5

    def fwd():
        N.check(N.fn("mdtf_attn_fwd")(N.ptr(qkv), N.ptr(mask), N.ptr(out), N.ptr(lse), B, S, nh, dh, scale, p, 99,
                                      None, N.stream_ptr()), "fwd")

    def bwd():
        N.check(N.fn("mdtf_attn_bwd")(N.ptr(qkv), N.ptr(mask), N.ptr(out), N.ptr(dout), N.ptr(lse), N.ptr(dqkv), B,
                                      S, nh, dh, scale, p, 99, None, N.stream_ptr()), "bwd")

    res = {0: {"fwd": [], "bwd": []}, 1: {"fwd": [], "bwd": []}}
    prev = N.fn("mdtf_set_attn_pp")(0)
    for rnd in range(5):
        for pp in (0, 1):
            N.fn("mdtf_set_attn_pp")(pp)
            fwd()
            tf = gtime(fwd) * 1000.0
            tb = gtime(bwd) * 1000.0
            res[pp]["fwd"].append(tf)
            res[pp]["bwd"].append(tb)
            print(json.dumps({"round": rnd, "pp": pp, "fwd_us": round(tf, 2), "bwd_us": round(tb, 2)}), flush=True)
    N.fn("mdtf_set_attn_pp")(prev)
    fl_f = 4.0 * B * nh * S * S * dh
    summ = {}
    for pp in (0, 1):
        f, b = statistics.median(res[pp]["fwd"]), statistics.median(res[pp]["bwd"])
        summ["pp%d" % pp] = {"fwd_us": round(f, 2), "bwd_us": round(b, 2), "fwd_TFs": round(fl_f / f / 1e6, 1),
                             "bwd_TFs": round(3.5 * fl_f / b / 1e6, 1)}
    print(json.dumps({"summary": summ, "B": B}), flush=True)


if __name__ == "__main__":
    main()
