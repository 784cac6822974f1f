#!/usr/bin/env python
"""Graph-timed residual + LayerNorm forward / backward kernels (csrc/transformer.hip) at BERT shapes.

Times ``mdtf_ln_fwd`` and ``mdtf_ln_bwd`` (+ its gamma / beta partial reduction) replayed back to back in a hipGraph
(the step runs them that way), prints one JSON line per shape with us/call and the streamed bytes' rate.  Env
switches of the kernels (MDTF_LN_BWD_RPB, ...) apply.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rows", type=int, nargs="+", default=[8192])
    p.add_argument("--H", type=int, default=768)
    p.add_argument("--p_drop", type=float, default=0.1)
    p.add_argument("--iters", type=int, default=50)
    a = p.parse_args()
    from mdtf.ops import _native as N
    from mdtf.ops import transformer as T  # noqa: F401  (registers the LN entry points)
    dev = torch.device("cuda", 0)
    for rows in a.rows:
        H = a.H
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(rows, H, device=dev, generator=g).bfloat16()
        r = torch.randn(rows, H, device=dev, generator=g).bfloat16()
        gamma = torch.rand(H, device=dev) + 0.5
        beta = torch.randn(H, device=dev)
        y, s = torch.empty_like(x), torch.empty_like(x)
        mean = torch.empty(rows, device=dev)
        rstd = torch.empty(rows, device=dev)
        dy = torch.randn(rows, H, device=dev, generator=g).bfloat16()
        ds, dxb = torch.empty_like(x), torch.empty_like(x)
        dgb = torch.zeros(2 * H, device=dev)
        ws = torch.empty(N.fn("mdtf_ln_bwd_ws")(rows, H), device=dev)
        off = torch.zeros(1, dtype=torch.int64, device=dev)

        def fwd():
            N.check(N.fn("mdtf_ln_fwd")(N.ptr(x), N.ptr(r), N.ptr(gamma), N.ptr(beta), N.ptr(y), N.ptr(s),
                                        N.ptr(mean), N.ptr(rstd), rows, H, 1e-12, a.p_drop, 1234, N.ptr(off),
                                        N.stream_ptr()), "ln_fwd")

        def bwd():
            N.check(N.fn("mdtf_ln_bwd")(N.ptr(dy), N.ptr(s), N.ptr(gamma), N.ptr(mean), N.ptr(rstd), N.ptr(ds),
                                        N.ptr(dxb), N.ptr(dgb), N.ptr(dgb[H:]), N.ptr(ws), rows, H, a.p_drop, 1234,
                                        N.ptr(off), N.stream_ptr()), "ln_bwd")

        out = {"rows": rows, "H": H, "p_drop": a.p_drop, "rpb": os.environ.get("MDTF_LN_BWD_RPB", "16")}
        for name, fn, nbytes in (("fwd", fwd, 4 * rows * H * 2), ("bwd", bwd, (4 if a.p_drop else 3) * rows * H * 2)):
            fn()
            torch.cuda.synchronize()
            st = torch.cuda.Stream(dev)
            with torch.cuda.stream(st):
                gr = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gr, stream=st):
                    for _ in range(a.iters):
                        fn()
            for _ in range(3):
                gr.replay()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for _ in range(5):
                e0.record()
                gr.replay()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / a.iters)
            t = sorted(ts)[len(ts) // 2]
            out[name + "_us"] = round(t, 2)
            out[name + "_TBps"] = round(nbytes / t / 1e6, 2)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
