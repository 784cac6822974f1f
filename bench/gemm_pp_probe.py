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


TILES = (0, 1, 2, 3, 4, 5)


def rnd(*shape):
    return (torch.rand(*shape, device="cuda") * 2 - 1).to(torch.bfloat16)


def rel_err(a, b):
    return float((a.float() - b.float()).abs().max() / (b.float().abs().max() + 1e-6))


def _try(fn):
    try:
        return fn()
    except RuntimeError as e:
        if "unsupported" in str(e):
            return None
        raise


def seg_check(M, Nn, K):
    """q|k|v-style segments: 2 weight matrices of Nn/2 columns in one launch, forward with bias + ReLU, data
    gradient with the ReLU backward from the saved pre-activation, weight gradient into two fp32 slots with the
    bias gradients, against fp32 torch."""
    ns = Nn // 2
    x = rnd(M, K)
    ws = [rnd(K, ns), rnd(K, ns)]
    bs = [rnd(ns), rnd(ns)]
    W = torch.cat(ws, 1).float()
    B = torch.cat(bs).float()
    pre = torch.empty(M, Nn, dtype=torch.bfloat16, device="cuda")
    y = mm.fwd(x, ws, biases=bs, act=1, pre=pre)
    ref_pre = x.float() @ W + B
    e = [rel_err(pre, ref_pre), rel_err(y, torch.relu(pre.float()))]
    dy = rnd(M, Nn)
    # dx = dy W^T (K-dim output); with act_bwd the product is multiplied by relu'(x) as if x were pre-activation
    dx = mm.dgrad(dy, ws)
    e.append(rel_err(dx, dy.float() @ W.t()))
    dxa = mm.dgrad(dy, ws, act_pre=x, act_bwd=1)
    e.append(rel_err(dxa, (dy.float() @ W.t()) * (x.float() > 0)))
    gws = [torch.zeros(K, ns, device="cuda") for _ in range(2)]
    dbs = [torch.zeros(ns, device="cuda") for _ in range(2)]
    ok = mm.wgrad_into(gws, x, dy, dbs=dbs)
    if ok:           # (the transposed operands need tile-aligned extents: K = 320 has no tile)
        gref = x.float().t() @ dy.float()
        e.append(rel_err(torch.cat(gws, 1), gref))
        e.append(rel_err(torch.cat(dbs), dy.float().sum(0)))
    good = max(e[:4]) < 2e-2 and max(e[4:] or [0.0]) < 1e-3 and (ok or K % 128 != 0)
    print(json.dumps({"seg_check": [M, Nn, K], "errs": [round(v, 6) for v in e], "ok": good}), flush=True)
    return good


def check():
    ok = True
    torch.manual_seed(0)
    shapes = [(520, 264, 192), (256, 256, 64), (1000, 776, 320), (128, 128, 128), (4096, 768, 768), (264, 1032, 704),
              (768, 2304, 512), (512, 768, 320)]
    for (M, Nn, K) in shapes:
        for tile in TILES:
            x, w = rnd(M, K), rnd(K, Nn)
            b = rnd(Nn)
            ref = x.float() @ w.float()
            y = mm.fwd(x, w, tile=tile)
            e0 = e1 = -1.0
            if y is not None:
                e0 = rel_err(y, ref)
                pre = torch.empty_like(y)
                yg = mm.fwd(x, w, biases=[b], act=2, pre=pre, tile=tile)
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
                gw = gw0.clone()
                if not mm.wgrad_into(gw, xt, dyt, tile=tile, splits=sp):
                    e4 = -1.0
                    break
                e4 = max(e4, rel_err(gw, wref))
            good = max(e0, e1, e2, e3) < 2e-2 and e4 < 1e-3 and e2 >= 0
            if tile == 5 and M % 128 == 0 and Nn % 192 == 0 and Nn >= 384:
                good &= seg_check(M, Nn, K)
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
        res = {"shape": name, "M": M, "N": Nn, "K": K}
        if not name.startswith("wg_"):
            x, w = rnd(M, K), rnd(K, Nn)
            wT = rnd(Nn, K)
            # forward y[M][Nn] = x w
            res["fwd_hipblaslt"] = gtime(lambda: torch.mm(x, w))
            for tile in TILES:
                if mm.fwd(x, w, tile=tile) is not None:
                    res["fwd_t%d" % tile] = gtime(lambda: mm.fwd(x, w, tile=tile))
            # data gradient with the same GEMM dims: C[M][Nn] = A[M][K] . W[Nn][K]^T  (W stored [Nn][K])
            res["dgrad_hipblaslt"] = gtime(lambda: torch.mm(x, wT.t()))
            for tile in TILES:
                res["dgrad_t%d" % tile] = gtime(lambda: mm.dgrad(x, wT, tile=tile))
            kinds = ("fwd", "dgrad")
        else:
            # weight gradient: C[M][Nn] (fp32) += X[K][M]^T . DY[K][Nn]  (K = tokens)
            xa, dya = rnd(K, M), rnd(K, Nn)
            gw = torch.zeros(M, Nn, device="cuda")
            res["wgrad_hipblaslt"] = gtime(lambda: torch.addmm(gw, xa.t(), dya, out_dtype=torch.float32, out=gw))
            for tile in TILES:
                if not mm.wgrad_into(gw, xa, dya, tile=tile, splits=1):
                    continue
                for sp in (1, 2, 3, 4, 6):
                    res["wgrad_t%d_s%d" % (tile, sp)] = gtime(lambda: mm.wgrad_into(gw, xa, dya, tile=tile, splits=sp))
            kinds = ("wgrad",)
        best = {k: v for k, v in res.items() if isinstance(v, float)}
        out = {k: (round(v * 1000, 2) if isinstance(v, float) else v) for k, v in res.items()}   # us
        for kind in kinds:
            mine = min((v, k) for k, v in best.items() if k.startswith(kind + "_t"))
            out[kind + "_best"] = mine[1]
            out[kind + "_best_tf"] = round(flops / mine[0] / 1e9, 1)
            out[kind + "_lib_tf"] = round(flops / best[kind + "_hipblaslt"] / 1e9, 1)
        print(json.dumps(out), flush=True)


BERT = [("qkv", 8192, 2304, 768), ("attn_out", 8192, 768, 768), ("ffn_in", 8192, 3072, 768),
        ("ffn_out", 8192, 768, 3072), ("wg_qkv", 768, 2304, 8192), ("wg_ffn_in", 768, 3072, 8192),
        ("wg_ffn_out", 3072, 768, 8192), ("wg_attn", 768, 768, 8192), ("dg_qkv", 8192, 768, 2304),
        ("dg_ffn_in", 8192, 768, 3072), ("dg_ffn_out", 8192, 3072, 768),
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
