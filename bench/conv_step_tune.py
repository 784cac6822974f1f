#!/usr/bin/env python
"""In-step conv tile selection: re-time the ResNet-50 training step with each convolution's candidate tiles.

``bench/conv_autotune.py`` times every candidate of a conv in isolation, where the operands stay resident in the
256 MB MALL across repetitions and the fused epilogues run without their in-step inputs (the pending residual
gradient, the BN-statistics operands).  Measured in the step (profiles/resnet_step_tune_r3.md) several choices
lose by 2x -- e.g. the stage-1 1x1 data gradient that folds the identity shortcut's gradient in.  This script
measures what the step actually costs:

1. runs the bench.py ResNet step eagerly and records every (pass, shape) that ``conv.choose`` resolves;
2. for each such conv, times all valid candidates in isolation (validity + a short list: the ``--top`` fastest
   of each kernel family);
3. swaps each short-listed candidate into the live table and times ``--steps`` whole training steps (CUDA
   events, after ``--warm`` steps), keeping a candidate only when it beats the current choice by more than the
   measured step-time noise twice in a row.

The tuned table goes to ``--out`` (copy it over mdtf/ops/conv_table.json after review) with a markdown report.
"""
import argparse
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from mdtf.ops import conv as C  # noqa: E402
import conv_autotune as T  # noqa: E402


def build_step(depth, batch):
    import mdtf
    from mdtf.data.loaders import SyntheticDataLoader
    from mdtf.models import ResNet, SoftmaxCrossEntropyLoss
    from mdtf.runtime import Net, Tower
    from mdtf.train import variables as V
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    store = V.get_store()
    store.device = dev
    store.compute_dtype = torch.bfloat16
    store.generator.manual_seed(1234)
    loader = SyntheticDataLoader(shape=(224, 224, 3), num_classes=1000, dtype=torch.bfloat16, seed=0)
    loader.batch_size = batch
    raw, gt = loader.load_train_batch()
    base = mdtf.train.MomentumOptimizer(0.1 * batch / 256.0, momentum=0.9, weight_decay=5e-5)
    gs = mdtf.train.get_or_create_global_step()
    tg = []
    Tower(Net(ResNet(depth)), "tower_0/", tg, raw, gt, SoftmaxCrossEntropyLoss(), base, batch_size=batch).process()
    opt = mdtf.train.SyncReplicasOptimizer(base, replicas_to_aggregate=1, total_num_replicas=1, hip_graph=False)
    op = opt.apply_gradients(T_avg(tg), global_step=gs)
    sess = mdtf.train.MonitoredTrainingSession(is_chief=True, checkpoint_dir=None, log_step_count_steps=0)
    return sess, op


def T_avg(tg):
    from mdtf.runtime import Tower
    return Tower.average_gradients(tg)


def step_ms(sess, op, steps, warm):
    for _ in range(warm):
        sess.run(op)
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(steps):
        sess.run(op)
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / steps


def parse_key(key):
    pass_, nhwc, k, s, p, d = key.split(":")
    n, h, w, c = map(int, nhwc.split(","))
    kh, kw, co = map(int, k.split(","))
    return pass_, (n, h, w, c), (kh, kw, c, co), tuple(map(int, s.split(","))), tuple(map(int, p.split(","))), \
        tuple(map(int, d.split(",")))


def candidates(pass_, xs, ws, stride):
    n, h, w, c = xs
    kh, kw, _, co = ws
    s = stride[0]
    out = []
    if pass_ in ("fwd", "dgrad"):
        if C.v2_ok(pass_, c, co, stride, kh * kw):
            out += [("v2", (bm, bn, 0, 2, st)) for bm, bn, st in T.V2_TILES]
            out += [("v3", (bm, bn, 0, 3, st)) for bm, bn, st in T.V3_TILES]
        out += [("ws", t) for t in T.ws_tiles(pass_, c, co, kh, kw, s)]
    else:
        if C.v2_ok("wgrad", c, co, stride, kh * kw):
            out += [("w2", (bm, bn, sp, 2, st)) for bm, bn, st in T.WG2_TILES for sp in (0, 16, 32, 64, 256, 2048)]
            out += [("w3", (bm, bn, sp, 3, st)) for bm, bn, st in T.WG3_TILES for sp in (0, 8, 16, 32, 64, 128, 1024)]
    return out


def entry(fam, cand):
    if fam == "ws":
        return {"backend": "mdtf", "ver": 4, "ws": list(cand)}
    bm, bn, sp, ver, st = cand
    return {"backend": "mdtf", "bm": bm, "bn": bn, "splits": sp, "ver": ver, "stages": st}


def same(e1, e2):
    keys = ("backend", "ver", "ws", "bm", "bn", "splits", "stages")
    return all(e1.get(k) == e2.get(k) for k in keys)


def iso_fn(pass_, xs, ws, stride, pads, dil, fam, cand, bufs):
    from mdtf.ops.padding import conv_geometry
    n, h, w, c = xs
    kh, kw, _, co = ws
    x, wt, dy, oh, ow = bufs
    if pass_ == "fwd":
        if fam == "ws":
            wtt = C.transpose_filter(wt)
            st = T._stats(co, 128, n * oh * ow)
            return lambda: C.ws_fwd(x, wtt, kh, kw, (oh, ow), stride, pads, dil, cand, st)
        bm, bn, sp, ver, stg = cand
        st = T._stats(co, bm, n * oh * ow)
        return lambda: C.mdtf_fwd(x, wt, (oh, ow), stride, pads, dil, bm, bn, st, ver, stg)
    if pass_ == "dgrad":
        if fam == "ws":
            return lambda: C.ws_dgrad(dy, wt, x.shape, pads, dil, cand)
        bm, bn, sp, ver, stg = cand
        return lambda: C.mdtf_dgrad(dy, wt, x.shape, stride, pads, dil, bm, bn, ver, stg)
    bm, bn, sp, ver, stg = cand
    return lambda: C.mdtf_wgrad(x, dy, wt.shape, stride, pads, dil, bm, bn, sp, None, ver, stg)


def dgrad_variants(xs, ws, stride, pads, dil, fam, cand, bufs):
    """The data gradient as the step runs it when it completes a BN output's gradient: BN-statistics epilogue
    plus a masked pending accumulate source (raises like the step would).  Returns the launch as a closure over
    its buffers, so it can also be timed."""
    x, wt, dy, oh, ow = bufs
    M = xs[0] * xs[1] * xs[2]
    mask = torch.full((M * xs[3] // 8,), 0x55, dtype=torch.uint8, device=x.device)
    g = torch.randn_like(x)
    out = torch.empty_like(x)
    if fam == "ws":
        st = T._stats(xs[3], 128, M)
        fn = lambda: C.ws_dgrad(dy, wt, x.shape, pads, dil, (2,) + tuple(cand[1:]), out=out,  # noqa: E731
                                bn_stats=(x, mask, st[0], st[1], st[0].shape[0]), acc_src=(g, mask))
    else:
        bm, bn, sp, ver, stg = cand
        st = T._stats(xs[3], bm, M)
        fn = lambda: C.mdtf_dgrad(dy, wt, x.shape, stride, pads, dil, bm, bn, ver, stg, out=out,  # noqa: E731
                                  bn_stats=(x, mask, st[0], st[1], st[0].shape[0]), acc_src=(g, mask))
    fn()
    return fn


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--depth", type=int, default=50)
    p.add_argument("--batch", type=int, default=256)
    p.add_argument("--steps", type=int, default=4)
    p.add_argument("--warm", type=int, default=1)
    p.add_argument("--top", type=int, default=3, help="isolated-fastest candidates kept per kernel family")
    p.add_argument("--passes", default="fwd,dgrad,wgrad")
    p.add_argument("--budget_s", type=float, default=900.0, help="stop trying new keys after this long")
    p.add_argument("--reverse", action="store_true", help="tune the keys last-seen first (continues a budget-capped "
                   "earlier run from the other end of the step)")
    p.add_argument("--rank_epilogue", action="store_true", help="short-list data-gradient tiles by their isolated "
                   "time WITH the BN-statistics + pending-accumulate epilogue (the plain launch ranks the small "
                   "tiles first, whose epilogue then costs the most in the step)")
    p.add_argument("--keys", default="", help="comma-free substrings: only tune keys containing one of them "
                   "(';'-separated)")
    p.add_argument("--out", default="gpurun_out/conv_table_step.json")
    p.add_argument("--report", default="gpurun_out/conv_step_tune.md")
    args = p.parse_args()
    t_start = time.time()
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    sess, op = build_step(args.depth, args.batch)
    seen = []
    real_choose = C.choose

    def rec(pass_, x_shape, w_shape, stride, pads, dil):
        k = C.shape_key(pass_, tuple(x_shape), tuple(w_shape), stride, pads, dil)
        if k not in seen:
            seen.append(k)
        return real_choose(pass_, x_shape, w_shape, stride, pads, dil)
    C.choose = rec
    for _ in range(3):
        sess.run(op)
    torch.cuda.synchronize()
    C.choose = real_choose
    table = C.table()
    keys = [k for k in seen if k in table and k.split(":")[0] in args.passes.split(",")
            and table[k].get("backend") == "mdtf"]
    if args.keys:
        keys = [k for k in keys if any(sub in k for sub in args.keys.split(";"))]
    if args.reverse:
        keys = keys[::-1]
    base = [step_ms(sess, op, args.steps, args.warm) for _ in range(6)]
    noise = statistics.pstdev(base)
    t0 = statistics.median(base)
    thr = max(2.5 * noise, 0.015)
    print("step %.3f ms (noise %.3f ms over %d), %d conv keys tuned in-step; threshold %.3f ms"
          % (t0, noise, len(base), len(keys), thr), flush=True)
    lines = ["| conv key | before | after | step ms before | step ms after | tried |", "|---|---|---|---:|---:|---:|"]
    changed = 0
    for key in keys:
        if time.time() - t_start > args.budget_s:
            print("budget reached; stopping before %s" % key, flush=True)
            break
        pass_, xs, ws, stride, pads, dil = parse_key(key)
        from mdtf.ops.padding import conv_geometry
        oh, ow, pt, pb, pl, pr = conv_geometry(xs[1], xs[2], ws[0], ws[1], stride, pads)
        x = torch.randn(*xs, device="cuda").bfloat16()
        wt = (torch.randn(*ws, device="cuda") * 0.05).bfloat16()
        dy = torch.randn(xs[0], oh, ow, ws[3], device="cuda").bfloat16()
        bufs = (x, wt, dy, oh, ow)
        fams = {}
        for fam, cand in candidates(pass_, xs, ws, stride):
            try:
                fn = iso_fn(pass_, xs, ws, stride, pads, dil, fam, cand, bufs)
                fn()
                if pass_ == "dgrad":          # the step's epilogue variants must take this tile too
                    fe = dgrad_variants(xs, ws, stride, pads, dil, fam, cand, bufs)
                    if args.rank_epilogue:    # short-list by the epilogue-carrying launch the step mostly runs
                        fn = fe
                torch.cuda.synchronize()
                t = T.timeit(fn, 3, warm=1)
            except RuntimeError:
                torch.cuda.synchronize()
                continue
            fams.setdefault(fam, []).append((t, cand))
        del x, wt, dy, bufs
        short = []
        for fam, lst in fams.items():
            for t, cand in sorted(lst)[:args.top]:
                short.append((fam, cand))
        cur = dict(table[key])
        t_cur = step_ms(sess, op, args.steps, args.warm)
        best = (t_cur, cur)
        tried = 0
        for fam, cand in short:
            e = entry(fam, cand)
            if same(e, cur):
                continue
            table[key] = e
            try:
                t = step_ms(sess, op, args.steps, args.warm)
            except RuntimeError as ex:        # a tile the step's epilogue variant does not take
                print("  %s %s failed in-step: %s" % (key, e, ex), flush=True)
                table[key] = cur
                torch.cuda.synchronize()
                raise
            tried += 1
            if t < best[0]:
                best = (t, e)
        table[key] = cur
        if best[1] is not cur and best[0] < t_cur - thr:
            # confirm: current vs best, interleaved
            table[key] = cur
            a = step_ms(sess, op, args.steps, args.warm)
            table[key] = best[1]
            b = step_ms(sess, op, args.steps, args.warm)
            if b < a - thr:
                e = dict(best[1])
                e["step_ms_gain"] = round(a - b, 4)
                table[key] = e
                changed += 1
                lines.append("| `%s` | %s | %s | %.3f | %.3f | %d |" % (
                    key, json.dumps({k: cur.get(k) for k in ("ver", "ws", "bm", "bn", "splits", "stages") if k in cur}),
                    json.dumps({k: e.get(k) for k in ("ver", "ws", "bm", "bn", "splits", "stages") if k in e}),
                    a, b, tried))
            else:
                table[key] = cur
        print("%s: %d tried, step %.3f -> %s" % (key, tried, t_cur, "%.3f %s" % (best[0], best[1])
                                                  if table[key] is not cur else "kept"), flush=True)
        with open(args.out, "w") as f:
            json.dump(table, f, indent=1, sort_keys=True)
    t1 = statistics.median([step_ms(sess, op, args.steps, args.warm) for _ in range(6)])
    with open(args.report, "w") as f:
        f.write("# In-step conv tile tuning (ResNet-%d, batch %d, eager step)\n\n" % (args.depth, args.batch))
        f.write("Step before: %.3f ms (noise %.3f ms); after %d changes: %.3f ms.\n\n" % (t0, noise, changed, t1))
        f.write("\n".join(lines) + "\n")
    print("step %.3f -> %.3f ms, %d changes" % (t0, t1, changed), flush=True)


if __name__ == "__main__":
    main()
