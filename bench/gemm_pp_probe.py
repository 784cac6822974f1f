"""Correctness + graph-timed speed of the ping-pong GEMM core (mdtf/csrc/gemm_pp.hip) against fp32 torch and
hipBLASLt (torch.mm), on random data.

  python bench/gemm_pp_probe.py --check          # numerics of every layout x tile (tails included)
  python bench/gemm_pp_probe.py                  # BERT-base / large shapes + square sizes, all tiles
Prints one JSON line per case.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from mdtf.ops import mm  # noqa: E402


def rnd(*shape):
    return (torch.rand(*shape, device="cuda") * 2 - 1).to(torch.bfloat16)


def rel_err(a, b):
    return float((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6))


def check():
    ok = True
    torch.manual_seed(0)
    shapes = [(520, 264, 192), (256, 256, 64), (1000, 776, 320), (128, 128, 128), (4096, 768, 768), (264, 1032, 704)]
    for (M, Nn, K) in shapes:
        for tile in (0, 1, 2, 3):
            x, w = rnd(M, K), rnd(K, Nn)
            b = rnd(Nn)
            ref = x.float() @ w.float()
            y = mm.fwd(x, w, tile=tile)
            e0 = rel_err(y, ref)
            pre = torch.empty_like(y)
            yg = mm.fwd(x, w, bias=b, act=2, pre=pre, tile=tile)
            refp = ref + b.float()
            refg = torch.nn.functional.gelu(refp.to(torch.bfloat16).float(), approximate="tanh")
            e1 = max(rel_err(pre, refp), rel_err(yg, refg))
            # dgrad with the same GEMM dims: dx [M, Nn] = dy [M, K] @ w2^T, w2 [Nn, K]
            dy, w2 = rnd(M, K), rnd(Nn, K)
            dref = dy.float() @ w2.float().t()
            dx = mm.dgrad(dy, w2, tile=tile)
            e2 = rel_err(dx, dref)
            acc0 = rnd(M, Nn)
            dxa = mm.dgrad(dy, w2, out=acc0.clone(), accumulate=True, tile=tile)
            e3 = rel_err(dxa, dref + acc0.float())
            # wgrad with the same GEMM dims: gw [M, Nn] += xt^T dyt, xt [K, M] (K tokens), dyt [K, Nn]
            xt, dyt = rnd(K, M), rnd(K, Nn)
            gw0 = torch.randn(M, Nn, device="cuda")
            wref = gw0 + xt.float().t() @ dyt.float()
            e4 = 0.0
            for sp in (1, 2):
                gw = mm.wgrad_into(gw0.clone(), xt, dyt, tile=tile, splits=sp)
                e4 = max(e4, rel_err(gw, wref))
            good = max(e0, e1, e2, e3) < 2e-2 and e4 < 1e-3
            ok &= good
            print(json.dumps({"check": [M, Nn, K], "tile": tile, "fwd": round(e0, 5), "fwd_bias_gelu": round(e1, 5),
                              "dgrad": round(e2, 5), "dgrad_acc": round(e3, 5), "wgrad": round(e4, 7),
                              "ok": good}), flush=True)
    return ok


def gtime(fn, reps=20, rounds=5):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps)
    ts.sort()
    return ts[len(ts) // 2]


def bench(shapes):
    for (name, M, Nn, K) in shapes:
        flops = 2.0 * M * Nn * K
        x, w = rnd(M, K), rnd(K, Nn)
        dy, wT = rnd(M, Nn), rnd(Nn, K)      # dgrad of a layer whose W is [Nn', K'] ... see below
        res = {"shape": name, "M": M, "N": Nn, "K": K}
        # forward y[M][Nn] = x w
        res["fwd_hipblaslt"] = gtime(lambda: torch.mm(x, w))
        for tile in (0, 1, 2, 3):
            res["fwd_t%d" % tile] = gtime(lambda: mm.fwd(x, w, tile=tile))
        # data gradient with the same GEMM dims: C[M][Nn] = A[M][K] . W[Nn][K]^T  (W stored [Nn][K])
        res["dgrad_hipblaslt"] = gtime(lambda: torch.mm(x, wT.t()))
        for tile in (0, 1, 2, 3):
            res["dgrad_t%d" % tile] = gtime(lambda: mm.dgrad(x, wT, tile=tile))
        # weight gradient with the same GEMM dims: C[M][Nn] (fp32) += X[K][M]^T . DY[K][Nn]
        xa, dya = rnd(K, M), rnd(K, Nn)
        gw = torch.zeros(M, Nn, device="cuda")
        res["wgrad_hipblaslt"] = gtime(lambda: torch.addmm(gw, xa.t(), dya, out_dtype=torch.float32, out=gw)
                                       if hasattr(torch, "addmm") else None)
        for tile in (0, 1, 2, 3):
            for sp in (1, 2, 4):
                res["wgrad_t%d_s%d" % (tile, sp)] = gtime(lambda: mm.wgrad_into(gw, xa, dya, tile=tile, splits=sp))
        best = {k: v for k, v in res.items() if isinstance(v, float)}
        out = {k: (round(v * 1000, 2) if isinstance(v, float) else v) for k, v in res.items()}   # us
        for kind in ("fwd", "dgrad", "wgrad"):
            mine = min(v for k, v in best.items() if k.startswith(kind + "_t"))
            out[kind + "_best_tf"] = round(flops / mine / 1e9, 1)
            out[kind + "_lib_tf"] = round(flops / best[kind + "_hipblaslt"] / 1e9, 1)
        print(json.dumps(out), flush=True)


BERT = [("qkv", 8192, 2304, 768), ("attn_out", 8192, 768, 768), ("ffn_in", 8192, 3072, 768),
        ("ffn_out", 8192, 768, 3072), ("wg_qkv", 768, 2304, 8192), ("wg_ffn_in", 768, 3072, 8192),
        ("wg_ffn_out", 3072, 768, 8192), ("wg_attn", 768, 768, 8192), ("dg_qkv", 8192, 768, 2304),
        ("sq4096", 4096, 4096, 4096), ("sq8192", 8192, 8192, 8192)]

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--shapes", default="")
    args = ap.parse_args()
    if args.check:
        sys.exit(0 if check() else 1)
    sel = [s for s in BERT if not args.shapes or s[0] in args.shapes.split(",")]
    bench(sel)
