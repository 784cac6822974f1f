#!/usr/bin/env python
"""Ping-pong conv kernel (csrc/gemm_pp.hip mdtf_conv_pp) vs the table's current choice, per ResNet-50 shape.

For every forward (with the fused BN statistics epilogue, as conv_bn runs it) and stride-1 data gradient of
ResNet-v1.5 at the given batch, time the backend ``conv_table.json`` picks today and each ping-pong tile, all
graph-timed (kernel time only, as inside the captured step), and check each candidate's output and statistics
against the current path.  One JSON line per (pass, shape) goes to ``--out``; ``--table`` merges the winners
into the conv table (``ver`` 5 entries) when they beat the current choice by ``--margin``.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench.conv_autotune import _stats, gtime, resnet_convs  # noqa: E402
from mdtf.ops import conv as C  # noqa: E402
from mdtf.ops.padding import conv_geometry  # noqa: E402


def _rel(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def current_fwd(ch, x, w, ohw, s, pads4, stats):
    if ch[0] == "ws":
        return C.ws_fwd(x, C.transpose_filter(w), w.shape[0], w.shape[1], ohw, (s, s), pads4, (1, 1), ch[1], stats)
    return C.mdtf_fwd(x, w, ohw, (s, s), pads4, (1, 1), ch[1], ch[2], stats, ch[4], ch[5])


def current_dgrad(ch, dy, w, xs, s, pads4):
    if ch[0] == "ws":
        return C.ws_dgrad(dy, w, xs, pads4, (1, 1), ch[1])
    return C.mdtf_dgrad(dy, w, xs, (s, s), pads4, (1, 1), ch[1], ch[2], ch[4], ch[5])


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--out", default="gpurun_out/conv_pp_probe.jsonl")
    p.add_argument("--passes", default="fwd,dgrad")
    p.add_argument("--table", action="store_true", help="merge winners into mdtf/ops/conv_table.json")
    p.add_argument("--margin", type=float, default=0.97, help="pp must take <= margin x the current time")
    args = p.parse_args()
    dev = torch.device("cuda")
    shapes, all_convs = resnet_convs(50, args.batch)
    counts = {sh: all_convs.count(sh) for sh in shapes}
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    fout = open(args.out, "w")
    table = C.table()
    new = {}
    tot = {"cur": 0.0, "best": 0.0}
    torch.manual_seed(0)
    for (n, h, w, c, kh, kw, co, s, pads) in shapes:
        if c % 8 or co % 8:
            continue
        x = torch.randn(n, h, w, c, device=dev).bfloat16()
        wt = (torch.randn(kh, kw, c, co, device=dev) / (kh * kw * c) ** 0.5).bfloat16()
        oh, ow, pt, pb, pl, pr = conv_geometry(h, w, kh, kw, (s, s), pads)
        pads4 = (pt, pb, pl, pr)
        dy = torch.randn(n, oh, ow, co, device=dev).bfloat16()
        flops = 2.0 * n * oh * ow * co * kh * kw * c
        for pass_ in args.passes.split(","):
            if not C.pp_ok(pass_, c, co, (s, s), kh, kw):
                continue
            key = C.shape_key(pass_, (n, h, w, c), (kh, kw, c, co), (s, s), pads4, (1, 1))
            ch = C.choose(pass_, (n, h, w, c), (kh, kw, c, co), (s, s), pads4, (1, 1))
            M = n * oh * ow if pass_ == "fwd" else n * h * w
            if pass_ == "fwd":
                st_ref = _stats(co, 128, M)
                ref = current_fwd(ch, x, wt, (oh, ow), s, pads4, st_ref)
                ref_s = st_ref[0].sum(0).clone()
                cur = (lambda st=_stats(co, 128, M): current_fwd(ch, x, wt, (oh, ow), s, pads4, st))
            else:
                ref = current_dgrad(ch, dy, wt, x.shape, s, pads4)
                cur = (lambda: current_dgrad(ch, dy, wt, x.shape, s, pads4))
            t_cur = gtime(cur, args.reps)
            rec = {"pass": pass_, "key": key, "count": counts[(n, h, w, c, kh, kw, co, s, pads)], "current": list(
                map(str, ch)), "cur_ms": round(t_cur, 4), "cur_tfs": round(flops / t_cur / 1e9), "pp": {}}
            best = None
            for tile in C.PP_TILES:
                if not C.pp_ok(pass_, c, co, (s, s), kh, kw, tile):
                    continue
                try:
                    if pass_ == "fwd":
                        st = _stats(co, C.PP_TILES[tile][0], M)
                        y = C.pp_fwd(x, wt, (oh, ow), (s, s), pads4, (1, 1), tile, st)
                        torch.cuda.synchronize()
                        err = max(_rel(y, ref), _rel(st[0].sum(0), ref_s))
                        fn = (lambda tile=tile, st=st: C.pp_fwd(x, wt, (oh, ow), (s, s), pads4, (1, 1), tile, st))
                    else:
                        y = C.pp_dgrad(dy, wt, x.shape, pads4, (1, 1), tile)
                        torch.cuda.synchronize()
                        err = _rel(y, ref)
                        fn = (lambda tile=tile: C.pp_dgrad(dy, wt, x.shape, pads4, (1, 1), tile))
                    t = gtime(fn, args.reps)
                except RuntimeError as e:
                    rec["pp"][tile] = {"error": str(e)[:120]}
                    torch.cuda.synchronize()
                    continue
                rec["pp"][tile] = {"ms": round(t, 4), "tfs": round(flops / t / 1e9), "rel_err": float("%.2e" % err)}
                if err < 2e-2 and (best is None or t < best[0]):
                    best = (t, tile)
            k = rec["count"]
            tot["cur"] += k * t_cur
            tot["best"] += k * min(t_cur, best[0] if best else 1e9)
            if best is not None and best[0] <= args.margin * t_cur:
                new[key] = {"backend": "mdtf", "ver": 5, "tile": best[1], "ms": round(best[0], 4),
                            "prev": table.get(key)}
                rec["choice"] = best[1]
            fout.write(json.dumps(rec) + "\n")
            fout.flush()
            print("%-5s %-40s x%d cur %.4f (%d TF/s) %s" % (pass_, key, k, t_cur, rec["cur_tfs"], " ".join(
                "t%s:%s" % (t, v.get("ms", "err")) for t, v in rec["pp"].items())), flush=True)
    print("per-step conv time of these passes: current %.3f ms, with the best pp tiles %.3f ms" %
          (tot["cur"], tot["best"]))
    fout.write(json.dumps({"summary": tot, "new": sorted(new)}) + "\n")
    if args.table and new:
        with open(C.TABLE_PATH) as f:
            merged = json.load(f)
        merged.update(new)
        with open(C.TABLE_PATH, "w") as f:
            json.dump(merged, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
