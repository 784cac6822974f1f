#!/usr/bin/env python
"""Extra v2 conv tiles vs the table's current choice, per ResNet-50 forward / data-gradient shape.

Graph-timed (kernel time only, as inside the captured step), each candidate checked against the current path's
output (and, for the forward, its fused BN statistics).  Winners (<= --margin x the current time) are merged into
``mdtf/ops/conv_table.json`` with ``--table``.  Default candidates: the 448 x 128 8-wave tile (``csrc/conv_igemm.hip``
dispatch_fd_v2w8), whose tile counts are 0.875 of a 256-CU wave where the 256-row tiles leave 0.77.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench.conv_autotune import _stats, gtime, resnet_convs  # noqa: E402
from bench.conv_pp_probe import _rel, current_dgrad, current_fwd  # noqa: E402
from mdtf.ops import conv as C  # noqa: E402
from mdtf.ops.padding import conv_geometry  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--out", default="gpurun_out/conv_tile_probe.jsonl")
    p.add_argument("--passes", default="fwd,dgrad")
    p.add_argument("--tiles", default="448:128:2:3,448:128:1:3", help="bm:bn:stages:ver,...")
    p.add_argument("--table", action="store_true", help="merge winners into mdtf/ops/conv_table.json")
    p.add_argument("--margin", type=float, default=0.98)
    p.add_argument("--cold", action="store_true",
                   help="evict L2 / Infinity Cache before every launch (a 384 MiB fill in the graph, its own time "
                        "subtracted): the step reads most conv operands cold, the back-to-back default reads them "
                        "from the 256 MiB Infinity Cache")
    args = p.parse_args()
    timer = gtime
    if args.cold:
        scr = torch.empty(384 << 20, dtype=torch.uint8, device="cuda")

        def flush():
            scr.fill_(1)
        base = gtime(flush, args.reps)

        def timer(fn, reps):
            def both():
                flush()
                fn()
            return gtime(both, reps) - base
    cands = [tuple(int(v) for v in t.split(":")) for t in args.tiles.split(",")]
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
        if c % 64 or co % 64:
            continue
        x = torch.randn(n, h, w, c, device=dev).bfloat16()
        wt = (torch.randn(kh, kw, c, co, device=dev) / (kh * kw * c) ** 0.5).bfloat16()
        oh, ow, pt, pb, pl, pr = conv_geometry(h, w, kh, kw, (s, s), pads)
        pads4 = (pt, pb, pl, pr)
        dy = torch.randn(n, oh, ow, co, device=dev).bfloat16()
        flops = 2.0 * n * oh * ow * co * kh * kw * c
        for pass_ in args.passes.split(","):
            key = C.shape_key(pass_, (n, h, w, c), (kh, kw, c, co), (s, s), pads4, (1, 1))
            ch = C.choose(pass_, (n, h, w, c), (kh, kw, c, co), (s, s), pads4, (1, 1))
            if ch[0] not in ("mdtf", "ws"):
                continue
            M = n * oh * ow if pass_ == "fwd" else n * h * w
            if pass_ == "fwd":
                st_ref = _stats(co, 128, M)
                ref = current_fwd(ch, x, wt, (oh, ow), s, pads4, st_ref)
                ref_s = st_ref[0].sum(0).clone()
                cur = (lambda st=_stats(co, 128, M): current_fwd(ch, x, wt, (oh, ow), s, pads4, st))
            else:
                ref = current_dgrad(ch, dy, wt, x.shape, s, pads4)
                cur = (lambda: current_dgrad(ch, dy, wt, x.shape, s, pads4))
            t_cur = timer(cur, args.reps)
            rec = {"pass": pass_, "key": key, "count": counts[(n, h, w, c, kh, kw, co, s, pads)],
                   "current": list(map(str, ch)), "cur_ms": round(t_cur, 4), "cur_tfs": round(flops / t_cur / 1e9),
                   "cands": {}}
            best = None
            for bm, bn, stg, ver in cands:
                tag = "%dx%d:s%d:v%d" % (bm, bn, stg, ver)
                try:
                    if pass_ == "fwd":
                        st = _stats(co, bm, M)
                        y = C.mdtf_fwd(x, wt, (oh, ow), (s, s), pads4, (1, 1), bm, bn, st, ver, stg)
                        torch.cuda.synchronize()
                        err = max(_rel(y, ref), _rel(st[0].sum(0), ref_s))
                        fn = (lambda bm=bm, bn=bn, stg=stg, ver=ver, st=st: C.mdtf_fwd(
                            x, wt, (oh, ow), (s, s), pads4, (1, 1), bm, bn, st, ver, stg))
                    else:
                        y = C.mdtf_dgrad(dy, wt, x.shape, (s, s), pads4, (1, 1), bm, bn, ver, stg)
                        torch.cuda.synchronize()
                        err = _rel(y, ref)
                        fn = (lambda bm=bm, bn=bn, stg=stg, ver=ver: C.mdtf_dgrad(
                            dy, wt, x.shape, (s, s), pads4, (1, 1), bm, bn, ver, stg))
                    t = timer(fn, args.reps)
                except RuntimeError as e:
                    rec["cands"][tag] = {"error": str(e)[:100]}
                    torch.cuda.synchronize()
                    continue
                rec["cands"][tag] = {"ms": round(t, 4), "tfs": round(flops / t / 1e9), "rel_err": float("%.2e" % err)}
                if err < 2e-2 and (best is None or t < best[0]):
                    best = (t, bm, bn, stg, ver)
            k = rec["count"]
            tot["cur"] += k * t_cur
            tot["best"] += k * min(t_cur, best[0] if best else 1e9)
            if best is not None and best[0] <= args.margin * t_cur:
                new[key] = {"backend": "mdtf", "bm": best[1], "bn": best[2], "stages": best[3], "ver": best[4],
                            "splits": 0, "ms": round(best[0], 4), "prev_ms": round(t_cur, 4)}
                rec["choice"] = new[key]
            fout.write(json.dumps(rec) + "\n")
            fout.flush()
            print("%-5s %-42s x%d cur %.4f %s" % (pass_, key, k, t_cur, " ".join(
                "%s:%s" % (t, v.get("ms", "err")) for t, v in rec["cands"].items())), flush=True)
    print("per-step time of these passes: current %.3f ms, with the winners %.3f ms (%d new entries)" %
          (tot["cur"], tot["best"], len(new)))
    fout.write(json.dumps({"summary": tot, "new": new}) + "\n")
    if args.table and new:
        with open(C.TABLE_PATH) as f:
            merged = json.load(f)
        merged.update(new)
        with open(C.TABLE_PATH, "w") as f:
            json.dump(merged, f, indent=1, sort_keys=True)
        print("merged %d entries into %s" % (len(new), C.TABLE_PATH))


if __name__ == "__main__":
    main()
