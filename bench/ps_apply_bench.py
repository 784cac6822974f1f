#!/usr/bin/env python
"""Async parameter-server apply throughput at BASELINE config 5 sizes (one MI355X, no communication).

Config 5 is ResNet-152 v1.5, 2 ps + 6 workers, batch 64 per worker (BASELINE.json; reference: PS placement
distribute_train.py:95-96,109-110, replicas_to_aggregate distribute_flags.py:26-29).  This builds ONE ps task's
share of the ResNet-152 variables (greedy by bytes over 2 tasks, as the async varspec splits them) in the PS's
grouped flat space (mdtf.parallel.async_ps._PSGroupedSpace) and times ``apply_batch``'s fused update
(``optimizer.update_multi``: k bf16 wire payloads applied as k consecutive momentum-SGD updates in one pass per
group, the weights' bf16 shadow refreshed once) for k = 1..6 payloads, CUDA-event timed, median of ``--reps``.

Reported: us per apply call and per update, and the ps's update capacity against the push rate of 6 workers whose
ResNet-152 batch-64 step takes ``--worker_ms`` (0: measured here as one eager synchronous training step of that
model on this GPU -- forward, backward and a local update, so slightly longer than an async worker's compute between
two pushes).
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def resnet_var_shapes(depth=152, width=64, classes=1000):
    """(name, shape, decay) of every trainable ResNet v1.5 variable (HWIO convs, BN gamma/beta, dense)."""
    from mdtf.models.resnet import DEPTHS
    out = []

    def conv_bn(name, cin, cout, k):
        out.append((name + "/weights", (k, k, cin, cout), True))
        out.append((name + "/BatchNorm/gamma", (cout,), False))
        out.append((name + "/BatchNorm/beta", (cout,), False))

    conv_bn("conv1", 3, width, 7)
    cin = width
    for s, n in enumerate(DEPTHS[depth]):
        f = width * 2 ** s
        for u in range(n):
            scope = "block%d/unit_%d/" % (s + 1, u + 1)
            if u == 0:
                conv_bn(scope + "shortcut", cin, 4 * f, 1)
            conv_bn(scope + "conv1", cin, f, 1)
            conv_bn(scope + "conv2", f, f, 3)
            conv_bn(scope + "conv3", f, 4 * f, 1)
            cin = 4 * f
    out.append(("logits/weights", (cin, classes), True))
    out.append(("logits/biases", (classes,), False))
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--num_ps", type=int, default=2)
    p.add_argument("--ps", type=int, default=0)
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--max_k", type=int, default=6)
    p.add_argument("--worker_ms", type=float, default=0.0, help="worker step time (0: measure it)")
    p.add_argument("--out", default="gpurun_out/ps_apply_bench.json")
    args = p.parse_args()
    from mdtf.parallel.async_ps import _PSGroupedSpace
    from mdtf.parallel.reducer import UpdateTarget
    from mdtf.train import variables as V
    from mdtf.train.optimizer import MomentumOptimizer
    dev = torch.device("cuda", 0)
    shapes = resnet_var_shapes()
    # greedy by bytes over the ps tasks (largest first), as a balanced device setter would place them
    load = [0] * args.num_ps
    task = {}
    for name, shp, _ in sorted(shapes, key=lambda t: -torch.Size(t[1]).numel()):
        k = min(range(args.num_ps), key=lambda i: load[i])
        task[name] = k
        load[k] += torch.Size(shp).numel()
    variables = []
    for name, shp, decay in shapes:
        if task[name] != args.ps:
            continue
        # BN affine and biases stay fp32 (no bf16 shadow), as the model's variables do
        v = V.Variable(name, torch.randn(shp, device=dev) * 0.01, trainable=True, keep_fp32=not decay)
        v.apply_weight_decay = decay
        v.ps_task = args.ps
        variables.append(v)
    space = _PSGroupedSpace(variables, dev, torch.bfloat16, args.num_ps)
    opt = MomentumOptimizer(0.1, 0.9, weight_decay=1e-4)
    numel = sum(g.numel for g in space.groups)
    payloads = [[torch.randn(g.numel, device=dev).to(torch.bfloat16 if g.shadow is not None else torch.float32)
                 for g in space.groups] for _ in range(args.max_k)]
    res = {"config": "ResNet-152 v1.5, %d ps, ps task %d" % (args.num_ps, args.ps), "params_this_ps": numel,
           "params_total": sum(load), "groups": len(space.groups), "wire": "bf16", "optimizer": "momentum 0.9 + wd",
           "apply": {}}
    for k in range(1, args.max_k + 1):
        def apply():
            with torch.no_grad():
                for gi, g in enumerate(space.groups):
                    opt.update_multi(UpdateTarget(g, g.master, g.grad, g.shadow, "full"),
                                     [payloads[i][gi] for i in range(k)], list(range(k)))
        for _ in range(3):
            apply()
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            apply()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b) * 1e3)
        us = statistics.median(ts)
        res["apply"][k] = {"us_per_apply": round(us, 1), "us_per_update": round(us / k, 1),
                           "GB_per_s_state": round(numel * 4 * 2 / (us * 1e-6) / 1e9, 1)}
        print("k=%d: %.1f us per apply, %.1f us per update" % (k, us, us / k), flush=True)
    wms = args.worker_ms
    if wms <= 0:
        wms = measure_worker(dev)
        res["worker_step_ms_measured"] = round(wms, 3)
    res["worker_step_ms"] = wms
    push_per_s = 6.0 / (wms * 1e-3)
    cap = {k: 1e6 / v["us_per_update"] for k, v in res["apply"].items()}
    res["push_rate_6_workers_per_s"] = round(push_per_s, 1)
    res["ps_update_capacity_per_s"] = {k: round(v, 1) for k, v in cap.items()}
    res["capacity_over_push_rate_k1"] = round(cap[1] / push_per_s, 2)
    res["capacity_over_push_rate_k6"] = round(cap[args.max_k] / push_per_s, 2)
    print(json.dumps(res))
    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump(res, f, indent=1)


def measure_worker(dev, batch=64, steps=5):
    """Forward + backward of ResNet-152 at batch 64 (the worker's compute between two pushes), median ms."""
    import mdtf
    from mdtf.models import ResNet, SoftmaxCrossEntropyLoss
    from mdtf.runtime import Net, Tower
    from mdtf.train import variables as V
    store = V.get_store()
    store.device = dev
    store.compute_dtype = torch.bfloat16
    xp = mdtf.placeholder(torch.float32, [None, 224, 224, 3])
    yp = mdtf.placeholder(torch.int64, [None])
    opt = mdtf.train.MomentumOptimizer(0.1, 0.9)
    tg = []
    t = Tower(Net(ResNet(152, num_classes=1000)), "tower_0/", tg, xp, yp, SoftmaxCrossEntropyLoss(), opt,
              batch_size=batch)
    _, loss, _ = t.process()
    op = opt.apply_gradients(Tower.average_gradients(tg), global_step=mdtf.train.get_or_create_global_step())
    sess = mdtf.train.MonitoredTrainingSession(log_step_count_steps=0)
    x = torch.randn(batch, 224, 224, 3)
    y = torch.randint(0, 1000, (batch,))
    ts = []
    for i in range(steps + 2):
        torch.cuda.synchronize()
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        sess.run([op, loss], feed_dict={xp: x, yp: y})
        b.record()
        b.synchronize()
        if i >= 2:
            ts.append(a.elapsed_time(b))
    return statistics.median(ts)


if __name__ == "__main__":
    main()
