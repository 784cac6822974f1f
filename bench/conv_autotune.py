#!/usr/bin/env python
"""Per-shape conv backend/tile selection on the MI355X (writes mdtf/ops/conv_table.json).

For every convolution of ResNet-v1.5 (depth/batch given) and each pass
(fwd / dgrad / wgrad) this times MIOpen and the hand-written implicit-GEMM
kernels at each tile configuration (CUDA events, median of ``--reps``
launches after warmup, all variants interleaved in one process) and records
the fastest.  A markdown summary with TFLOP/s per shape goes to ``--report``.
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdtf.ops import conv as C  # noqa: E402
from mdtf.ops import winograd as Wg  # noqa: E402
from mdtf.ops.padding import conv_geometry  # noqa: E402


def resnet_convs(depth=50, batch=256, image=224, width=64):
    from mdtf.models.resnet import DEPTHS
    blocks = DEPTHS[depth]
    out = []
    h = image
    out.append((batch, h, h, 3, 7, 7, width, 2, (3, 3, 3, 3)))
    h = h // 2
    h = (h + 1) // 2  # maxpool 3x3/2 SAME
    cin = width
    for s, n in enumerate(blocks):
        f = width * 2 ** s
        for u in range(n):
            stride = 2 if (u == 0 and s > 0) else 1
            if u == 0:
                out.append((batch, h, h, cin, 1, 1, 4 * f, stride, (0, 0, 0, 0)))
            out.append((batch, h, h, cin, 1, 1, f, 1, (0, 0, 0, 0)))
            if stride == 1:
                out.append((batch, h, h, f, 3, 3, f, 1, (1, 1, 1, 1)))
            else:
                out.append((batch, h, h, f, 3, 3, f, 2, (1, 1, 1, 1)))
            h2 = (h + 2 - 3) // stride + 1
            out.append((batch, h2, h2, f, 1, 1, 4 * f, 1, (0, 0, 0, 0)))
            h = h2
            cin = 4 * f
    uniq = []
    for c in out:
        if c not in uniq:
            uniq.append(c)
    return uniq, out


WG2_TILES = ((128, 128, 2), (128, 128, 3), (128, 128, 4), (128, 128, 5), (128, 64, 2), (64, 128, 2), (64, 128, 4),
             (64, 128, 6), (64, 64, 3))
WG3_TILES = ((256, 256, 2), (256, 128, 2), (256, 128, 3), (128, 256, 2), (128, 256, 3), (128, 128, 3), (128, 128, 4),
             (128, 128, 5), (64, 256, 3), (64, 256, 4), (256, 64, 3), (256, 64, 4))   # 8 waves
# (bm, bn, stages): LDS = stages * (bm + bn) * 128 B <= 160 KiB
V2_TILES = ((128, 128, 2), (128, 128, 3), (128, 128, 4), (128, 64, 3), (128, 64, 4), (256, 128, 2), (256, 128, 3),
            (256, 64, 3), (64, 128, 2), (64, 128, 3), (64, 128, 4), (64, 64, 4),
            (128, 128, 1), (128, 64, 1), (256, 128, 1), (64, 128, 1), (256, 64, 1),   # stages 1: K == 64 only
            (128, 128, 32), (64, 128, 32), (64, 128, 42))   # split rings: 10 x A stages + filter stages
# 8-wave (512-thread) v2 tiles: one block per CU, 2 waves per SIMD
V3_TILES = ((256, 256, 2), (256, 128, 2), (256, 128, 3), (256, 64, 3), (256, 64, 4), (128, 256, 2), (128, 256, 3),
            (256, 256, 1), (256, 128, 1), (448, 128, 2), (448, 128, 1),   # 448 = 7 x 64: 0.875-wave tile counts
            (256, 256, 32), (256, 128, 32), (256, 128, 42), (128, 256, 32), (128, 256, 42))   # split rings


def ws_tiles(pass_, c, co, kh, kw, s):
    """Weight-stationary kernel tiles (csrc/conv_ws.hip) valid for this conv pass."""
    if not C.ws_ok(pass_, c, co, (s, s), kh, kw):
        return []
    red, ncol = (c, co) if pass_ == "fwd" else (co, c)
    kt = kh * kw * red
    out = []
    for tp in (2, 4):
        for nw in (4, 8):
            for cg in (1, 2, 4):
                if nw % cg or ncol % (64 * cg) or cg * kt * 128 > 160 * 1024:
                    continue
                for d in (2, 3, 4, 6):
                    if C.ws_depth_ok(kt, d):
                        out.append((tp, nw, cg, d))
    return out


def _stats(co, bm, M):
    """Statistics buffer as conv_bn uses it (slot count as in ops/conv.py)."""
    import torch
    mtiles = -(-M // bm)
    slots = C.STAT_SLOTS
    while slots < 1024 and slots * 8 < mtiles:
        slots *= 2
    buf = torch.zeros((2, slots, co), dtype=torch.float32, device="cuda")
    return (buf[0], buf[1])


GRAPH = [False]     # --graph: time the mdtf candidates inside captured graphs (kernel time only, as in the step)


def gtime(fn, reps, warm=3):
    """Kernel time per launch: ``reps`` launches captured into one graph, median of 5 replays."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) / reps)
    del g
    return statistics.median(ts)


def timeit(fn, reps, warm=3, graph=False):
    if graph:
        return gtime(fn, reps, warm)
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--depth", type=int, default=50)
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--reps", type=int, default=10)
    p.add_argument("--out", default=C.TABLE_PATH)
    p.add_argument("--report", default="gpurun_out/conv_autotune.md")
    p.add_argument("--passes", default="fwd,dgrad,wgrad")
    p.add_argument("--strides", default="", help="only shapes with these strides (e.g. 2)")
    p.add_argument("--merge", action="store_true", help="update the existing table at --out instead of replacing it")
    p.add_argument("--graph", action="store_true",
                   help="time the mdtf and Winograd candidates inside captured graphs (no host launch cost)")
    p.add_argument("--step_epilogues", action="store_true",
                   help="dgrad: time every candidate with the epilogue the training step runs -- the BN-backward "
                        "statistics of the gradient it completes, plus (block inputs: 1x1 stride-1 convs narrowing "
                        "the channels) the masked identity-shortcut gradient folded in; adds the ping-pong core")
    args = p.parse_args()
    GRAPH[0] = args.graph
    dev = torch.device("cuda")
    shapes, all_convs = resnet_convs(args.depth, args.batch)
    counts = {s: all_convs.count(s) for s in shapes}
    table = {}
    lines = ["| pass | shape (N,H,W,C,k,Co,s) | count | miopen ms | best mdtf ms (tile) | winograd ms | TF/s mdtf |"
             " choice |", "|---|---|---|---|---|---|---|---|"]
    tot = {"miopen": 0.0, "best": 0.0}
    torch.manual_seed(0)
    if args.strides:
        keep = {int(v) for v in args.strides.split(",")}
        shapes = [sh for sh in shapes if sh[7] in keep]
    for (n, h, w, c, kh, kw, co, s, pads) in shapes:
        x = torch.randn(n, h, w, c, device=dev).bfloat16()
        wt = (torch.randn(kh, kw, c, co, device=dev) * 0.05).bfloat16()
        oh, ow, pt, pb, pl, pr = conv_geometry(h, w, kh, kw, (s, s), (pads[0], pads[1], pads[2], pads[3]))
        pads4 = (pt, pb, pl, pr)
        dy = torch.randn(n, oh, ow, co, device=dev).bfloat16()
        flops = 2.0 * n * oh * ow * co * kh * kw * c
        native_ok = c % 8 == 0 and co % 8 == 0
        for pass_ in args.passes.split(","):
            key = C.shape_key(pass_, (n, h, w, c), (kh, kw, c, co), (s, s), pads4, (1, 1))
            if pass_ == "fwd":
                lib = lambda: C.miopen_fwd(x, wt, (s, s), pads4, (1, 1))  # noqa: E731
                cands = [(bm, bn, 0, 1) for bm, bn in ((128, 128), (128, 64), (64, 64), (256, 64))]
                if C.v2_ok("fwd", c, co, (s, s), kh * kw):
                    cands += [(bm, bn, st, 2) for bm, bn, st in V2_TILES]
                    cands += [(bm, bn, st, 3) for bm, bn, st in V3_TILES]
                cands += [(t, 0, 0, 4) for t in ws_tiles("fwd", c, co, kh, kw, s)]
                wtt = C.transpose_filter(wt)

                if args.step_epilogues:
                    cands += [(t, 0, 0, 5) for t in C.PP_TILES if C.pp_ok("fwd", c, co, (s, s), kh, kw, t)]

                # training always runs conv -> BN: time the forward with its fused statistics epilogue
                def mk(bm, bn, sp, v):
                    if v == 5:
                        st = _stats(co, C.PP_TILES[bm][0], n * oh * ow)
                        return lambda: C.pp_fwd(x, wt, (oh, ow), (s, s), pads4, (1, 1), bm, st)
                    if v == 4:
                        st = _stats(co, 128, n * oh * ow)
                        return lambda: C.ws_fwd(x, wtt, kh, kw, (oh, ow), (s, s), pads4, (1, 1), bm, st)
                    st = _stats(co, bm, n * oh * ow)
                    return lambda: C.mdtf_fwd(x, wt, (oh, ow), (s, s), pads4, (1, 1), bm, bn, st, v, sp)
            elif pass_ == "dgrad":
                lib = lambda: C.miopen_bwd(x, wt, dy, (s, s), pads4, (1, 1), True, False)  # noqa: E731
                cands = [(bm, bn, 0, 1) for bm, bn in ((128, 128), (128, 64), (64, 64), (256, 64))]
                if C.v2_ok("dgrad", c, co, (s, s), kh * kw):
                    cands += [(bm, bn, st, 2) for bm, bn, st in V2_TILES]
                    cands += [(bm, bn, st, 3) for bm, bn, st in V3_TILES]
                cands += [(t, 0, 0, 4) for t in ws_tiles("dgrad", c, co, kh, kw, s)]

                if args.step_epilogues:
                    cands = [cd for cd in cands if cd[3] != 1]          # v1: no statistics epilogue
                    cands += [(t, 0, 0, 5) for t in C.PP_TILES if C.pp_ok("dgrad", c, co, (s, s), kh, kw, t)]
                    bx = torch.randn(n, h, w, c, device=dev).bfloat16()
                    mbits = torch.randint(0, 256, (n * h * w * c // 8,), device=dev, dtype=torch.uint8)
                    sb = torch.zeros(2, C.STAT_SLOTS, c, device=dev)
                    bst = (bx, mbits, sb[0], sb[1], C.STAT_SLOTS)
                    block_in = kh == 1 and s == 1 and c > co
                    pend = (torch.randn(n, h, w, c, device=dev).bfloat16(), mbits) if block_in else None
                    dxb = torch.empty(n, h, w, c, device=dev, dtype=torch.bfloat16)

                    def mk(bm, bn, sp, v):
                        if v == 4:
                            return lambda: C.ws_dgrad(dy, wt, x.shape, pads4, (1, 1), (2,) + tuple(bm[1:]), out=dxb,
                                                      bn_stats=bst, acc_src=pend)
                        if v == 5:
                            return lambda: C.pp_dgrad(dy, wt, x.shape, pads4, (1, 1), bm, out=dxb, bn_stats=bst,
                                                      acc_src=pend)
                        return lambda: C.mdtf_dgrad(dy, wt, x.shape, (s, s), pads4, (1, 1), bm, bn, v, sp, out=dxb,
                                                    bn_stats=bst, acc_src=pend)
                else:
                    def mk(bm, bn, sp, v):
                        if v == 4:
                            return lambda: C.ws_dgrad(dy, wt, x.shape, pads4, (1, 1), bm)
                        return lambda: C.mdtf_dgrad(dy, wt, x.shape, (s, s), pads4, (1, 1), bm, bn, v, sp)
            else:
                lib = lambda: C.miopen_bwd(x, wt, dy, (s, s), pads4, (1, 1), False, True)  # noqa: E731
                cands = [(bm, bn, sp, 1) for bm, bn in ((128, 128), (64, 64), (128, 64), (64, 128))
                         for sp in (0, 256, 2048)]
                if C.v2_ok("wgrad", c, co, (s, s), kh * kw):
                    # splits: 0 = ~4 (4-wave) / ~2 (8-wave) blocks per CU; fewer splits = longer pixel runs
                    # per block and fewer fp32 atomics per output element
                    cands += [((bm, st), bn, sp, 2) for bm, bn, st in WG2_TILES for sp in (0, 16, 32, 64, 256, 2048)]
                    cands += [((bm, st), bn, sp, 3) for bm, bn, st in WG3_TILES for sp in (0, 8, 16, 32, 64, 128, 1024)]
                mk = lambda bm, bn, sp, v: (lambda: C.mdtf_wgrad(  # noqa
                    x, dy, wt.shape, (s, s), pads4, (1, 1), bm[0] if v >= 2 else bm, bn, sp, None, v,
                    bm[1] if v >= 2 else 2))
            t_lib = timeit(lib, args.reps)
            t_wino = None
            if pass_ in ("fwd", "dgrad") and Wg.eligible((kh, kw), (s, s), pads4, (1, 1), c, co):
                wfn = ((lambda: Wg.winograd_fwd(x, wt, (oh, ow), pads4)) if pass_ == "fwd"
                       else (lambda: Wg.winograd_dgrad(dy, wt, x.shape, pads4)))
                try:
                    t_wino = timeit(wfn, args.reps, graph=GRAPH[0])
                except RuntimeError:
                    t_wino = timeit(wfn, args.reps)
            best = None
            best_np = None                                   # best candidate outside the ping-pong core
            second = {}
            if native_ok:
                for bm, bn, sp, v in cands:
                    try:
                        t = timeit(mk(bm, bn, sp, v), args.reps, graph=GRAPH[0])
                    except RuntimeError:
                        torch.cuda.synchronize()
                        continue
                    if best is None or t < best[0]:
                        best = (t, bm, bn, sp, v)
                    if v != 5 and (best_np is None or t < best_np[0]):
                        best_np = (t, bm, bn, sp, v)
            if best_np is not None:
                t0, bm0, bn0, sp0, v0 = best_np
                if v0 == 4:
                    second[pass_] = {"backend": "mdtf", "ver": 4, "ws": list(bm0), "ms": round(t0, 4)}
                else:
                    second[pass_] = {"backend": "mdtf", "bm": bm0, "bn": bn0, "splits": 0, "ver": v0,
                                     "stages": sp0, "ms": round(t0, 4)}
            if t_wino is not None and t_wino < t_lib and (best is None or t_wino < best[0]):
                table[key] = {"backend": "winograd", "ms": round(t_wino, 4), "miopen_ms": round(t_lib, 4),
                              "mdtf_ms": round(best[0], 4) if best else None}
                choice = "winograd"
            # a library forward cannot fuse the following BatchNorm's statistics (a separate pass over y),
            # which the mdtf timing includes; a library dgrad cannot accumulate into a fanned-out input's
            # gradient or emit the BN backward statistics in its epilogue (an extra add / reduction pass):
            # MIOpen must be clearly faster to be chosen for either
            elif best is not None and best[0] < {"fwd": t_lib / 0.85, "dgrad": t_lib / 0.75}.get(pass_, t_lib):
                ent = {"backend": "mdtf", "bm": best[1], "bn": best[2], "splits": best[3], "ver": best[4],
                       "ms": round(best[0], 4), "miopen_ms": round(t_lib, 4)}
                if best[4] == 4:                          # weight-stationary kernel: tile in "ws"
                    ent = {"backend": "mdtf", "ver": 4, "ws": list(best[1]), "ms": round(best[0], 4),
                           "miopen_ms": round(t_lib, 4)}
                elif best[4] == 5:                        # ping-pong core: tile index, "prev" = best of the rest
                    ent = {"backend": "mdtf", "ver": 5, "tile": best[1], "ms": round(best[0], 4),
                           "miopen_ms": round(t_lib, 4)}
                    rest = second[pass_] if second.get(pass_) else None
                    if rest is not None:
                        ent["prev"] = rest
                elif best[4] >= 2 and pass_ == "wgrad":   # v2 wgrad: bm field carries (rows, stages)
                    ent["bm"], ent["stages"] = best[1]
                elif best[4] in (2, 3):                   # v2 fwd/dgrad: the third field is the pipeline depth
                    ent["stages"], ent["splits"] = best[3], 0
                table[key] = ent
                choice = "mdtf"
            else:
                table[key] = {"backend": "miopen", "ms": round(t_lib, 4),
                              "mdtf_ms": round(best[0], 4) if best else None}
                choice = "miopen"
            k = counts[(n, h, w, c, kh, kw, co, s, pads)]
            tot["miopen"] += k * t_lib
            tot["best"] += k * min(t_lib, best[0] if best else 1e9, t_wino or 1e9)
            lines.append("| %s | %d,%d,%d,%d,%dx%d,%d,s%d | %d | %.3f | %s | %s | %s | %s |" % (
                pass_, n, h, w, c, kh, kw, co, s, k, t_lib,
                ("%.3f (%s,%s,%s,v%d)" % best) if best else "n/a",
                ("%.3f" % t_wino) if t_wino is not None else "-",
                ("%.0f" % (flops / best[0] / 1e9)) if best else "-", choice))
            print(lines[-1], flush=True)
    lines.append("")
    lines.append("Total conv time per training step (sum over passes x occurrences): MIOpen %.2f ms, "
                 "best-of %.2f ms" % (tot["miopen"], tot["best"]))
    print(lines[-1])
    if args.merge and os.path.exists(args.out):
        with open(args.out) as f:
            merged = json.load(f)
        merged.update(table)
        table = merged
    with open(args.out, "w") as f:
        json.dump(table, f, indent=1, sort_keys=True)
    os.makedirs(os.path.dirname(args.report) or ".", exist_ok=True)
    with open(args.report, "w") as f:
        f.write("# Conv autotune (ResNet-%d, batch %d, bf16, MI355X)\n\n" % (args.depth, args.batch))
        f.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
