#!/usr/bin/env python
"""BASELINE config 5: ResNet-152 asynchronous parameter-server training, 2 ps + 6 workers on one node.

Parent mode (no --job_name): starts the whole localhost ClusterSpec (ps tasks on
GPUs 0..P-1, worker tasks on the next GPUs: one process per GPU, RankLayout's
async-PS device order), waits, and prints one JSON line with the aggregate
worker throughput (images/sec summed over workers, measured by each worker
after its warmup steps).

Task mode (--job_name/--task_index given, reference CLI): a reference-style
annotated ``main`` (as distribute.py) with ResNet-152 v1.5, synthetic
ImageNet-shaped data, momentum SGD and ``ps_mode='async'``.

Needs num_ps + num_workers GPUs (default 8): the round-end driver runs it on an
8-GPU node; on a CPU host use --cpu with a small --depth/--image for plumbing.
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--num_ps", type=int, default=2)
    p.add_argument("--num_workers", type=int, default=6)
    p.add_argument("--model", choices=("resnet", "bert"), default="resnet",
                   help="bert: BERT pre-training (tied, vocabulary-padded MLM decoder) under the async PS")
    p.add_argument("--bert_size", default="tiny")
    p.add_argument("--seq", type=int, default=128)
    p.add_argument("--depth", type=int, default=152)
    p.add_argument("--batch", type=int, default=64)
    p.add_argument("--image", type=int, default=224)
    p.add_argument("--steps", type=int, default=30, help="timed steps per worker")
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--cpu", action="store_true", help="plumbing run on the CPU (gloo)")
    p.add_argument("--share_gpu", action="store_true", help="all tasks on GPU 0, gloo transport (1-GPU rehearsal)")
    p.add_argument("--timeout_s", type=float, default=1800)
    return p.parse_known_args(argv)


def parent(a):
    from mdtf.cluster.launcher import launch_local_cluster
    out = tempfile.mkdtemp(prefix="mdtf_async_bench_")
    env = {"MDTF_BENCH_OUT": out, "MDTF_BENCH_WARMUP": str(a.warmup), "HSA_ENABLE_IPC_MODE_LEGACY": "0"}
    if a.cpu:
        env["CUDA_VISIBLE_DEVICES"] = ""
        env["HIP_VISIBLE_DEVICES"] = ""
    elif a.share_gpu:
        # every task on the one visible GPU, tensors exchanged over gloo (RCCL needs a device per rank): the
        # 1-GPU rehearsal of the async data plane, not a throughput measurement of config 5
        env["MDTF_DIST_BACKEND"] = "gloo"
    argv = [os.path.abspath(__file__), "--depth=%d" % a.depth, "--batch=%d" % a.batch, "--image=%d" % a.image,
            "--steps=%d" % a.steps, "--warmup=%d" % a.warmup, "--ps_mode=async", "--model=%s" % a.model,
            "--bert_size=%s" % a.bert_size, "--seq=%d" % a.seq]
    t0 = time.time()
    codes = launch_local_cluster(argv, a.num_ps, a.num_workers, extra_env=env, timeout_s=a.timeout_s)
    wall = time.time() - t0
    if any(codes):
        print(json.dumps({"error": "task exit codes %s" % codes}))
        return 1
    rates, stale = [], []
    for i in range(a.num_workers):
        with open(os.path.join(out, "worker%d.json" % i)) as f:
            r = json.load(f)
        rates.append(r["steps"] * r["batch"] / max(r["seconds"], 1e-9))
    value = sum(rates)
    ps_stats = []
    for p in range(a.num_ps):
        fn = os.path.join(out, "ps%d.json" % p)
        if os.path.exists(fn):
            with open(fn) as f:
                ps_stats.append(json.load(f))
    print(json.dumps({
        "metric": "%s async parameter-server, %d ps + %d workers, one node" % (
            ("sequences/sec BERT-%s" % a.bert_size) if a.model == "bert" else ("images/sec ResNet-%d" % a.depth),
            a.num_ps, a.num_workers),
        "value": round(value, 2), "unit": "sequences/sec" if a.model == "bert" else "images/sec", "n_gpus": 0 if a.cpu else (1 if a.share_gpu else a.num_ps + a.num_workers),
        "higher_is_better": True, "per_worker": [round(x, 2) for x in rates], "wall_s": round(wall, 1),
        "ps": [{k: r.get(k) for k in ("ps", "updates", "mean_staleness", "max_staleness", "apply_s", "idle_s", "wall_s",
                                      "store_wait_s", "store_calls", "applies", "batched_max", "poll", "wire")}
               for r in ps_stats],
        "dtype": "bf16" if not a.cpu else "fp32", "data": "synthetic", "config": {
            "model": ("bert-%s seq%d" % (a.bert_size, a.seq)) if a.model == "bert" else "resnet%d_v1.5" % a.depth, "per_worker_batch": a.batch, "image": a.image,
            "parallelism": "async-ps %dps+%dw" % (a.num_ps, a.num_workers)}}), flush=True)
    return 0


def task(a):
    import mdtf
    from mdtf.config import annotations
    from mdtf.config.flags import FLAGS
    from mdtf.data.loaders import SyntheticDataLoader
    from mdtf.models import ResNet, SoftmaxCrossEntropyLoss
    from mdtf.runtime.entry import run_from_annotations

    from mdtf.models import Bert, BertPretrainingLoss, SyntheticBertLoader

    class BenchResNet(ResNet):
        def __init__(self):
            super(BenchResNet, self).__init__(a.depth)

    class BenchLoader(SyntheticDataLoader):
        def __init__(self):
            super(BenchLoader, self).__init__(shape=(a.image, a.image, 3), num_classes=1000)

    class BenchBert(Bert):
        def __init__(self):
            super(BenchBert, self).__init__(a.bert_size, seq_len=a.seq)

    class BenchBertLoader(SyntheticBertLoader):
        def __init__(self):
            super(BenchBertLoader, self).__init__(a.seq, seed=FLAGS.task_index)

    class BenchBertLoss(BertPretrainingLoss):
        def __init__(self):
            super(BenchBertLoss, self).__init__()

    for c in (BenchResNet, BenchLoader, SoftmaxCrossEntropyLoss, BenchBert, BenchBertLoader, BenchBertLoss):
        annotations.register_class(c)
    total = (a.warmup + a.steps) * a.num_workers
    bert = a.model == "bert"
    opt = (mdtf.train.AdamOptimizer(1e-4) if bert else mdtf.train.MomentumOptimizer(0.1 * a.batch / 256, 0.9))

    @annotations.current_model(model="BenchBert" if bert else "BenchResNet")
    @annotations.optimizer(optimizer=opt)
    @annotations.loss(loss="BenchBertLoss" if bert else "SoftmaxCrossEntropyLoss")
    @annotations.current_mode(mode="Train")
    @annotations.current_input(input="BenchBertLoader" if bert else "BenchLoader")
    @annotations.gpu_num(gpu_num=1)
    @annotations.job_name(job_name=FLAGS.job_name)
    @annotations.task_index(task_index=FLAGS.task_index)
    @annotations.batch_size(batch_size=a.batch)
    @annotations.sample_number(sample_number=total * a.batch)
    @annotations.epoch_num(epoch_num=1)
    @annotations.ps_mode(ps_mode="async")
    def main(argv):
        return run_from_annotations(main, module=sys.modules[__name__])

    return main(sys.argv)


if __name__ == "__main__":
    args, rest = parse()
    if any(r.startswith("--job_name") for r in rest):
        from mdtf.config.flags import FLAGS
        FLAGS(sys.argv[:1] + rest)
        sys.exit(task(args) or 0)
    sys.exit(parent(args))
