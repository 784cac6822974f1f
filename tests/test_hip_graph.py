"""hipGraph-captured training steps (mdtf.train.graph) == eager steps.

Deterministic mode makes every cross-block reduction fixed-order, so a
replayed graph must reproduce the eager run bit for bit: same inputs copied
into the static buffers, same per-step LR / Adam bias correction read from the
device hyper-parameter buffer.
"""
import os

import pytest
import torch

import mdtf
from mdtf.ops import optim


class _TinyRes(object):
    def inference(self, x):
        from mdtf.layers import tools
        from mdtf.ops import nn as ops
        from mdtf.train import variables as V
        store = V.get_store()
        if store.compute_dtype is not None:
            x = x.to(store.compute_dtype)
        s = tools.conv_bn("c1", x, 64, 3, 1, relu=True)
        y = tools.conv_bn("c2", s, 64, 1, 1, relu=True)
        x = tools.conv_bn("c3", y, 64, 3, 1, relu=True, residual=s)
        x = tools.conv_bn("c4", x, 128, 3, 2, relu=True)
        x = ops.global_avg_pool(x)
        return tools.dense("logits", x, 16)


def _run_resnetish(dev, dt, batches, hip_graph, opt_kind="momentum", mode="allreduce"):
    from mdtf.models import SoftmaxCrossEntropyLoss
    from mdtf.runtime import Model, Net, Tower
    from mdtf.train import step as S
    from mdtf.train import variables as V
    V.reset_default_graph()
    S.reset()
    store = V.get_store()
    store.device = torch.device(dev)
    store.compute_dtype = dt
    store.generator.manual_seed(7)
    x0, _ = batches[0]
    xp = mdtf.placeholder(torch.float32, [None] + list(x0.shape[1:]))
    yp = mdtf.placeholder(torch.int64, [None])
    if opt_kind == "momentum":
        base = mdtf.train.MomentumOptimizer(lambda step: 0.05 / (1 + step), 0.9, weight_decay=1e-4)
    else:
        base = mdtf.train.AdamOptimizer(1e-3)
    tg = []
    M = type("TinyResModel", (_TinyRes, Model), {})
    t = Tower(Net(M()), "tower_0/", tg, xp, yp, SoftmaxCrossEntropyLoss(), base, batch_size=x0.shape[0])
    _, loss, _ = t.process()
    opt = mdtf.train.SyncReplicasOptimizer(base, hip_graph=hip_graph, mode=mode, bucket_bytes=1 << 18)
    op = opt.apply_gradients(Tower.average_gradients(tg), global_step=mdtf.train.get_or_create_global_step())
    sess = mdtf.train.MonitoredTrainingSession(log_step_count_steps=0)
    losses = []
    for x, y in batches:
        _, lv = sess.run([op, loss], feed_dict={xp: x, yp: y})
        losses.append(lv)
    losses = [float(v) for v in losses]        # fetched tensors must keep their step's value
    weights = {v.name: v.value().detach().float().cpu().clone() for v in store.trainable_variables()}
    return losses, weights, op


def test_optimizer_dyn_buffer_cpu_reference():
    """The device hyper-parameter buffer overrides lr / lr_t / grad scale (torch reference path)."""
    torch.manual_seed(0)
    w = torch.randn(64)
    g = torch.randn(64)
    a, b = w.clone(), w.clone()
    acc_a, acc_b = torch.zeros(64), torch.zeros(64)
    optim.momentum_(a, g, acc_a, None, 0.1, 0.9, 0.5, 0.0)
    optim.momentum_(b, g, acc_b, None, 99.0, 0.9, 7.0, 0.0, dyn=torch.tensor([0.1, 0.1, 0.5]))
    assert torch.equal(a, b)
    ma, va, mb, vb = (torch.zeros(64) for _ in range(4))
    a, b = w.clone(), w.clone()
    optim.adam_(a, g, ma, va, None, 1e-3, 0.9, 0.999, 1e-8, 3, 0.5)
    lr_t = optim.adam_lr_t(1e-3, 0.9, 0.999, 3)
    optim.adam_(b, g, mb, vb, None, 5.0, 0.9, 0.999, 1e-8, 1, 3.0, dyn=torch.tensor([1e-3, lr_t, 0.5]))
    assert torch.allclose(a, b, rtol=1e-6, atol=1e-9)


def test_hip_graph_flag_falls_back_to_eager_on_cpu():
    torch.manual_seed(0)
    batches = [(torch.randn(4, 8, 8, 3), torch.randint(0, 16, (4,))) for _ in range(3)]
    l_e, w_e, _ = _run_resnetish("cpu", None, batches, hip_graph=False)
    l_g, w_g, op = _run_resnetish("cpu", None, batches, hip_graph=True)
    assert l_e == l_g
    assert op.graph is None or op.graph.graph is None
    for k in w_e:
        assert torch.equal(w_e[k], w_g[k]), k


def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mdtf.ops import _native
    _native.lib()


@pytest.mark.gpu
@pytest.mark.parametrize("opt_kind", ["momentum", "adam"])
def test_hip_graph_step_bitwise_equals_eager(opt_kind):
    _gpu()
    from mdtf.ops import _native
    torch.manual_seed(0)
    batches = [(torch.randn(16, 16, 16, 8), torch.randint(0, 16, (16,))) for _ in range(6)]
    _native.set_deterministic(True)
    try:
        l_e, w_e, _ = _run_resnetish("cuda", torch.bfloat16, batches, hip_graph=False, opt_kind=opt_kind)
        l_g, w_g, op = _run_resnetish("cuda", torch.bfloat16, batches, hip_graph=True, opt_kind=opt_kind)
    finally:
        _native.set_deterministic(False)
    g = op.graph
    assert g is not None and g.graph is not None and g.replays == 4 and g.fallbacks == 0, vars(g)
    assert l_e == l_g, (l_e, l_g)
    for k in w_e:
        assert torch.equal(w_e[k], w_g[k]), k


@pytest.mark.gpu
def test_hip_graph_shape_change_falls_back():
    _gpu()
    torch.manual_seed(0)
    batches = [(torch.randn(8, 16, 16, 8), torch.randint(0, 16, (8,))) for _ in range(4)]
    batches.append((torch.randn(4, 16, 16, 8), torch.randint(0, 16, (4,))))   # a short last batch
    batches.append((torch.randn(8, 16, 16, 8), torch.randint(0, 16, (8,))))
    l_g, _, op = _run_resnetish("cuda", torch.bfloat16, batches, hip_graph=True)
    assert op.graph.fallbacks == 1 and op.graph.replays == 3
    assert all(v == v for v in l_g)


@pytest.mark.gpu
def test_hip_graph_capture_failure_stays_eager(monkeypatch):
    """A capture the runtime rejects does not abort training: that step and every later one run eagerly."""
    _gpu()
    from mdtf.train import graph as G

    def boom(self, ctx, step):
        raise RuntimeError("operation not permitted when stream is capturing")
    monkeypatch.setattr(G.StepGraph, "_capture", boom)
    torch.manual_seed(0)
    batches = [(torch.randn(8, 16, 16, 8), torch.randint(0, 16, (8,))) for _ in range(5)]
    l_g, _, op = _run_resnetish("cuda", torch.bfloat16, batches, hip_graph=True)
    assert op.graph.disabled and op.graph.graph is None and op.graph.replays == 0
    assert len(l_g) == 5 and all(v == v for v in l_g)


@pytest.mark.gpu
def test_hip_graph_bert_dropout_advances_per_replay():
    """BERT-tiny with dropout under graph replay: the device step counter advances every replay (fresh
    dropout masks), the loss keeps decreasing, and every replay is a real step."""
    _gpu()
    from mdtf.models import Bert, BertPretrainingLoss, SyntheticBertLoader
    from mdtf.runtime import Net, Tower
    from mdtf.train import graph as G
    from mdtf.train import variables as V
    store = V.get_store()
    store.device = torch.device("cuda")
    store.compute_dtype = torch.bfloat16
    rng0 = int(G.rng_offset_tensor(store.device).item())
    ld = SyntheticBertLoader(seq_len=128, max_predictions=5, vocab=1000)
    ld.batch_size = 8
    raw, gt = ld.load_train_batch()
    base = mdtf.train.AdamWeightDecayOptimizer(1e-3)
    tg = []
    model = Bert("tiny", vocab_size=1000, seq_len=128, max_predictions=5, dropout=0.1)
    model.heads = model.H // 64       # head dim 64: the fused attention kernel (with dropout) runs
    t = Tower(Net(model), "tower_0/", tg, raw, gt, BertPretrainingLoss(5), base, batch_size=8)
    _, loss, _ = t.process()
    opt = mdtf.train.SyncReplicasOptimizer(base, hip_graph=True)
    op = opt.apply_gradients(Tower.average_gradients(tg), global_step=mdtf.train.get_or_create_global_step())
    sess = mdtf.train.MonitoredTrainingSession(log_step_count_steps=0)
    ls = []
    for _ in range(25):
        _, lv = sess.run([op, loss])
        ls.append(lv)
    ls = [float(v) for v in ls]
    assert op.graph.replays == 23
    assert int(G.rng_offset_tensor(store.device).item()) - rng0 == 23
    assert len(set(ls[3:])) > 10          # not the same masked step replayed over and over
    assert sum(ls[-5:]) < 0.7 * sum(ls[:5]), ls


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["allreduce", "sharded", "sharded-inline"])
def test_hip_graph_captures_rccl_collectives(mode, monkeypatch):
    """The bucketed RCCL all-reduce (or PS-shard reduce-scatter + all-gather) fired from the gradient hooks
    is captured into the step graph: a 1-rank nccl group with collectives forced on, eager == replay.

    Sharded: inside the capture bucket k's update (and all-gather) is issued when bucket k+1
    launches, the last one in end_backward, so the backward kernels captured between hook k and hook k+1 do not
    depend on bucket k's reduce-scatter (``capture_update_log``: bucket k updated once k+2 buckets had launched).
    ``sharded-inline`` is the round-5 order (update inside the bucket's own hook).  The side-stream form
    (MDTF_SHARDED_CAPTURE_UPD=fork) segfaults in hipStreamEndCapture on this ROCm and is not run."""
    _gpu()
    from mdtf.parallel import reducer as R
    inline = mode == "sharded-inline"
    mode = "sharded" if inline else mode
    monkeypatch.setattr(R.GradReducer, "CAPTURE_UPD", "inline" if inline else "lag")
    import socket
    import torch.distributed as dist
    from mdtf.ops import _native
    monkeypatch.setenv("MDTF_FORCE_COLLECTIVES", "1")
    monkeypatch.setenv("TORCH_FR_BUFFER_SIZE", "2000")          # capture drains the watchdog by state
    # an intermittent abort from a non-Python thread after capture (r2, ~1 in 5 full-suite runs) printed no cause:
    # RCCL's own warnings name the failing call next time
    monkeypatch.setenv("NCCL_DEBUG", os.environ.get("NCCL_DEBUG", "WARN"))
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1)
    try:
        torch.manual_seed(0)
        batches = [(torch.randn(16, 16, 16, 8), torch.randint(0, 16, (16,))) for _ in range(5)]
        _native.set_deterministic(True)
        try:
            l_e, w_e, op_e = _run_resnetish("cuda", torch.bfloat16, batches, hip_graph=False, mode=mode)
            l_g, w_g, op = _run_resnetish("cuda", torch.bfloat16, batches, hip_graph=True, mode=mode)
        finally:
            _native.set_deterministic(False)
        assert op_e.reducer.collective and op_e.reducer.overlap and len(op_e.space.buckets) > 1
        assert op.graph.replays == 3 and op.graph.fallbacks == 0
        if mode == "sharded":
            # every bucket was updated + all-gathered during backward INSIDE the capture (not after the update)
            assert getattr(op.reducer, "captured_bucket_updates", 0) == len(op.space.buckets), \
                (getattr(op.reducer, "captured_bucket_updates", 0), len(op.space.buckets))
            nb = len(op.space.buckets)
            log = op.reducer.capture_update_log[-nb:]          # the capture's step
            assert [b for b, _ in log] == list(range(nb)) or sorted(b for b, _ in log) == list(range(nb)), log
            if not inline:
                # bucket k updated after bucket k+1 launched (the last after every bucket launched)
                assert all(launched >= min(k + 2, nb) for k, (_, launched) in enumerate(log)), log
        from mdtf.train import graph as G
        assert G.LAST_DRAIN[0] == "recorder", G.LAST_DRAIN
        assert l_e == l_g, (l_e, l_g)
        for k in w_e:
            assert torch.equal(w_e[k], w_g[k]), k
    finally:
        from mdtf.train import step as S
        S.release_graphs()                 # the captured RCCL collectives go before their communicator
        dist.destroy_process_group()


@pytest.mark.gpu
def test_drain_waits_for_watchdog_retirement(monkeypatch):
    """Capture starts only after the RCCL watchdog RETIRED every eager work (flight-recorder ``retired``),
    not merely after the device finished it: an eager all-reduce is still held by the watchdog right after
    synchronize(), and the drain returns only once it is gone."""
    _gpu()
    import socket
    import torch.distributed as dist
    from mdtf.train import graph as G
    monkeypatch.setenv("TORCH_FR_BUFFER_SIZE", "2000")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1)
    try:
        t = torch.ones(1 << 16, device="cuda")
        for _ in range(3):
            dist.all_reduce(t)
        torch.cuda.synchronize()
        ents = G._recorder_entries()
        assert ents, "flight recorder must be on for the drain"
        wm = max(e["record_id"] for e in ents)
        held_before = len(G._unretired(ents, wm))
        got = G._drain_comm_watchdog(timeout_s=30.0)
        assert got == wm and G.LAST_DRAIN[0] == "recorder"
        assert G._unretired(G._recorder_entries(), wm) == []
        # the watchdog loop sleeps between polls, so right after synchronize() it normally still holds the works
        # (held_before > 0) and the drain polls until they are retired; the watchdog may also retire them between
        # that sample and the drain's first look (a round-6 suite run saw held_before = 3 and no poll), so the
        # poll count is reported, not asserted -- the invariant is the line above: nothing unretired at return
        assert held_before >= 0 and G.LAST_DRAIN_POLLS[0] >= 0
    finally:
        dist.destroy_process_group()
