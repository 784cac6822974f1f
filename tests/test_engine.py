"""Variable store, step engine, sessions, hooks, optimizers (single process, CPU)."""
import math

import numpy as np
import pytest
import torch

import mdtf
from mdtf.data.loaders import SyntheticDataLoader
from mdtf.layers import tools
from mdtf.models import LeNet, SoftmaxCrossEntropyLoss
from mdtf.runtime import Loss, Model, Net, Tower
from mdtf.train import hooks as H
from mdtf.train import step as S
from mdtf.train import variables as V


def test_variable_scopes_and_reuse():
    with V.variable_scope("a"):
        w = V.get_variable("w", [2, 3], initializer=V.constant_initializer(1.0))
        with pytest.raises(ValueError):
            V.get_variable("w", [2, 3])
    with V.variable_scope("a", reuse=True):
        w2 = V.get_variable("w", [2, 3])
    assert torch.equal(w, w2)
    with V.variable_scope("a", reuse=V.AUTO_REUSE):
        V.get_variable("w", [2, 3])
        V.get_variable("new", [1])
    names = [v.name for v in V.global_variables()]
    assert names == ["a/w", "a/new"]
    with V.variable_scope("b", reuse=True):
        with pytest.raises(ValueError):
            V.get_variable("missing", [1])


def test_collections_scoped():
    with V.name_scope("tower_0"):
        V.add_to_collection("losses", torch.tensor(1.0))
    with V.name_scope("tower_1"):
        V.add_to_collection("losses", torch.tensor(2.0))
    assert len(V.get_collection("losses")) == 2
    assert float(V.get_collection("losses", "tower_1")[0]) == 2.0


def test_tools_variable_names():
    x = torch.randn(2, 8, 8, 3)
    with torch.no_grad():
        y = tools.conv("conv1", x, 3, 4)
        y = tools.conv_nonacti("conv2", y, 4, 4)
        y = tools.pool("p", y)
        y = tools.norm("n", y)
        y = tools.FC_layer("fc", y, 5)
        d = tools.deconv("dc", torch.randn(2, 4, 4, 6), 3, 6, output_shape=[2, 8, 8, 3], stride=[1, 2, 2, 1])
    names = [v.name for v in V.global_variables()]
    assert names == ["conv1/weights", "conv1/biases", "conv2/weights_nonacti", "conv2/biases_nonacti",
                     "fc/weights", "fc/biases", "dc/weights"]
    assert y.shape == (2, 5) and d.shape == (2, 8, 8, 3)
    assert V.get_store().vars["fc/weights"].shape == (4 * 4 * 4, 5)


def test_legacy_batch_norm_matches_reference():
    x = torch.randn(4, 3, 3, 2)
    y = tools.batch_norm(x, legacy=True)
    m = x.mean(0)
    v = x.var(0, unbiased=False)
    assert torch.allclose(y, (x - m) / torch.sqrt(v + 1e-3), atol=1e-5)


class _Linear(Model):
    def inference(self, x):
        w = V.get_variable("w", [4, 1], initializer=V.constant_initializer(0.0))
        b = V.get_variable("b", [1], initializer=V.constant_initializer(0.0))
        return x @ w + b


class _MSE(Loss):
    def loss(self, p, t):
        return ((p - t) ** 2).mean()


def _linear_problem(opt, steps=200, batch=32):
    torch.manual_seed(0)
    true_w = torch.tensor([[1.0], [-2.0], [0.5], [3.0]])
    xs = torch.randn(batch, 4)
    ys = xs @ true_w + 0.25
    x_ph = mdtf.placeholder(torch.float32, [None, 4])
    y_ph = mdtf.placeholder(torch.float32, [None, 1])
    tg = []
    gs = mdtf.train.get_or_create_global_step()
    tower = Tower(Net(_Linear()), "tower_0/", tg, x_ph, y_ph, _MSE(), opt, batch_size=batch)
    _, loss, _ = tower.process()
    train_op = opt.apply_gradients(Tower.average_gradients(tg), global_step=gs)
    with mdtf.train.MonitoredTrainingSession(hooks=[mdtf.train.StopAtStepHook(last_step=steps)],
                                             log_step_count_steps=0) as sess:
        while not sess.should_stop():
            _, step, lv = sess.run([train_op, gs, loss], feed_dict={x_ph: xs, y_ph: ys})
    return lv, step, V.get_store()


@pytest.mark.parametrize("opt", [lambda: mdtf.train.GradientDescentOptimizer(0.1),
                                 lambda: mdtf.train.MomentumOptimizer(0.05, 0.9),
                                 lambda: mdtf.train.AdamOptimizer(0.05)])
def test_optimizers_converge(opt):
    lv, step, store = _linear_problem(opt())
    assert step == 200
    assert lv < 1e-3
    assert abs(store.vars["w"].master[1, 0].item() + 2.0) < 0.05


def test_session_fetch_structures_and_global_step():
    lv, step, store = _linear_problem(mdtf.train.GradientDescentOptimizer(0.1), steps=5)
    assert step == 5 and mdtf.train.get_global_step().value() == 5


def test_forward_only_fetch_does_not_train():
    x_ph = mdtf.placeholder(torch.float32, [None, 4])
    y_ph = mdtf.placeholder(torch.float32, [None, 1])
    opt = mdtf.train.GradientDescentOptimizer(0.1)
    tg = []
    tower = Tower(Net(_Linear()), "tower_0/", tg, x_ph, y_ph, _MSE(), opt, batch_size=4)
    _, loss, logits = tower.process()
    opt.apply_gradients(Tower.average_gradients(tg), global_step=mdtf.train.get_or_create_global_step())
    sess = mdtf.train.MonitoredTrainingSession(log_step_count_steps=0)
    xs, ys = torch.ones(4, 4), torch.ones(4, 1)
    out = sess.run({"loss": loss, "logits": logits}, feed_dict={x_ph: xs, y_ph: ys})
    assert out["loss"] == pytest.approx(1.0) and out["logits"].shape == (4, 1)
    assert mdtf.train.get_global_step().value() == 0
    with pytest.raises(KeyError):
        sess.run(loss)


def test_step_counter_examples_hook_and_summaries(tmp_path):
    loader = SyntheticDataLoader(shape=(28, 28, 1), num_classes=10)
    loader.batch_size = 8
    raw, gt = loader.load_train_batch()
    opt = mdtf.train.AdamOptimizer(1e-3)
    gs = mdtf.train.get_or_create_global_step()
    tg = []
    tower = Tower(Net(LeNet()), "tower_0/", tg, raw, gt, SoftmaxCrossEntropyLoss(), opt, batch_size=8)
    _, loss, _ = tower.process()
    train_op = opt.apply_gradients(Tower.average_gradients(tg), global_step=gs)
    eps = H.ExamplesPerSecondHook(batch_size=8, every_n_steps=2)
    nan = H.NanTensorHook(loss)
    with mdtf.train.MonitoredTrainingSession(checkpoint_dir=str(tmp_path), hooks=[H.StopAtStepHook(num_steps=6), eps, nan],
                                             save_summaries_steps=2, log_step_count_steps=2,
                                             save_checkpoint_secs=None, save_checkpoint_steps=3) as sess:
        while not sess.should_stop():
            sess.run(train_op)
    assert eps.average_examples_per_sec and eps.average_examples_per_sec > 0
    from mdtf.utils import summary
    import glob
    ev = glob.glob(str(tmp_path / "events.out.tfevents.*"))
    assert ev
    tags = {t for _, t, _ in summary.read_events(ev[0])}
    assert "total_loss" in tags
    assert mdtf.train.latest_checkpoint(str(tmp_path)).endswith("model.ckpt-6")


def test_checkpoint_restore_resumes(tmp_path):
    def build():
        V.reset_default_graph()
        S.reset()
        loader = SyntheticDataLoader(shape=(28, 28, 1), num_classes=10)
        loader.batch_size = 4
        raw, gt = loader.load_train_batch()
        opt = mdtf.train.MomentumOptimizer(0.01, 0.9)
        gs = mdtf.train.get_or_create_global_step()
        tg = []
        tower = Tower(Net(LeNet()), "tower_0/", tg, raw, gt, SoftmaxCrossEntropyLoss(), opt, batch_size=4)
        _, loss, _ = tower.process()
        return opt.apply_gradients(Tower.average_gradients(tg), global_step=gs), gs
    train_op, gs = build()
    with mdtf.train.MonitoredTrainingSession(checkpoint_dir=str(tmp_path), hooks=[H.StopAtStepHook(last_step=4)],
                                             log_step_count_steps=0, save_checkpoint_secs=None,
                                             save_checkpoint_steps=4) as sess:
        while not sess.should_stop():
            sess.run(train_op)
    w_saved = V.get_store().vars["fc2/weights"].master.clone()
    mom_saved = train_op.space.groups[0].state_buffer("full/momentum").clone()
    train_op, gs = build()
    assert not torch.equal(V.get_store().vars["fc2/weights"].master, w_saved)
    with mdtf.train.MonitoredTrainingSession(checkpoint_dir=str(tmp_path), hooks=[H.StopAtStepHook(last_step=4)],
                                             log_step_count_steps=0, save_checkpoint_secs=None) as sess:
        assert sess.should_stop()          # already at last_step after restore
    assert gs.value() == 4
    assert torch.equal(V.get_store().vars["fc2/weights"].master, w_saved)
    assert torch.equal(train_op.space.groups[0].state_buffer("full/momentum"), mom_saved)


def test_weight_decay_collection_and_fused_decay_equivalent():
    # l2 loss in the 'losses' collection == optimizer-fused decay (grad += wd * w)
    torch.manual_seed(0)
    x = torch.randn(8, 4)
    y = torch.randn(8, 1)

    def run(fused):
        V.reset_default_graph()
        S.reset()
        x_ph, y_ph = mdtf.placeholder(torch.float32, [None, 4]), mdtf.placeholder(torch.float32, [None, 1])

        class M(Model):
            def inference(self, inp):
                w = V.get_variable("w", [4, 1], initializer=V.constant_initializer(0.5))
                if not fused:
                    V.add_to_collection("losses", mdtf.nn.l2_loss(w) * 0.1)
                return inp @ w
        opt = mdtf.train.GradientDescentOptimizer(0.1, weight_decay=0.1 if fused else 0.0)
        tg = []
        t = Tower(Net(M()), "tower_0/", tg, x_ph, y_ph, _MSE(), opt, batch_size=8)
        t.process()
        op = opt.apply_gradients(Tower.average_gradients(tg), global_step=mdtf.train.get_or_create_global_step())
        sess = mdtf.train.MonitoredTrainingSession(log_step_count_steps=0)
        for _ in range(3):
            sess.run(op, feed_dict={x_ph: x, y_ph: y})
        return V.get_store().vars["w"].master.clone()
    assert torch.allclose(run(True), run(False), atol=1e-6)


def test_learning_rate_json_and_schedules(tmp_path):
    from mdtf.utils.learning_rate import LearningRate, piecewise_constant, warmup_linear_decay
    p = str(tmp_path / "lr.json")
    lr = LearningRate(0.1, p, decay_factor=0.5)
    assert lr.learning_rate == 0.1
    lr.update(0.05)
    assert LearningRate(0.1, p).learning_rate == 0.05
    assert lr.decay() == 0.025
    f = piecewise_constant([10, 20], [1.0, 0.1, 0.01])
    assert (f(0), f(15), f(25)) == (1.0, 0.1, 0.01)
    g = warmup_linear_decay(1.0, 10, 110)
    assert g(0) == pytest.approx(0.1) and g(60) == pytest.approx(0.5)


def test_device_setter_round_robin():
    from mdtf.train.device_setter import replica_device_setter
    setter = replica_device_setter(cluster={"ps": ["a:1", "b:2"], "worker": ["c:3"]})
    with V.device(setter):
        for i in range(5):
            V.get_variable("v%d" % i, [1])
    assert [V.get_store().vars["v%d" % i].ps_task for i in range(5)] == [0, 1, 0, 1, 0]


def test_checkpoint_relative_model_dir_resume_and_cleanup(tmp_path, monkeypatch):
    """--model_dir=ck (relative): the state file stores paths relative to ck/, resume finds the
    latest checkpoint, and max_to_keep deletes the old shards (checkpoint_state.py)."""
    import glob
    import os
    monkeypatch.chdir(tmp_path)

    def build():
        V.reset_default_graph()
        S.reset()
        loader = SyntheticDataLoader(shape=(28, 28, 1), num_classes=10)
        loader.batch_size = 4
        raw, gt = loader.load_train_batch()
        opt = mdtf.train.MomentumOptimizer(0.01, 0.9)
        gs = mdtf.train.get_or_create_global_step()
        tg = []
        tower = Tower(Net(LeNet()), "tower_0/", tg, raw, gt, SoftmaxCrossEntropyLoss(), opt, batch_size=4)
        tower.process()
        return opt.apply_gradients(Tower.average_gradients(tg), global_step=gs), gs
    train_op, gs = build()
    saver = mdtf.train.Saver(max_to_keep=2)
    scaffold = mdtf.train.Scaffold(saver=saver)
    with mdtf.train.MonitoredTrainingSession(checkpoint_dir="ck", hooks=[H.StopAtStepHook(last_step=8)],
                                             scaffold=scaffold, log_step_count_steps=0, save_checkpoint_secs=None,
                                             save_checkpoint_steps=2) as sess:
        while not sess.should_stop():
            sess.run(train_op)
    txt = open(os.path.join("ck", "checkpoint")).read()
    assert 'model_checkpoint_path: "model.ckpt-8"' in txt and "ck/" not in txt
    assert sorted(os.path.basename(p) for p in glob.glob("ck/*.index")) == ["model.ckpt-6.index",
                                                                          "model.ckpt-8.index"]
    assert mdtf.train.latest_checkpoint("ck").endswith("model.ckpt-8")
    w_saved = V.get_store().vars["fc2/weights"].master.clone()
    train_op, gs = build()
    with mdtf.train.MonitoredTrainingSession(checkpoint_dir="ck", hooks=[H.StopAtStepHook(last_step=8)],
                                             log_step_count_steps=0, save_checkpoint_secs=None):
        pass
    assert gs.value() == 8
    assert torch.equal(V.get_store().vars["fc2/weights"].master, w_saved)


def test_conv_table_lookup_is_batch_agnostic():
    """Shapes at other batches (ResNet-152 async PS at batch 64) take the batch-256 tuned entries."""
    from mdtf.ops import conv as C
    w = (1, 1, 64, 256)
    a = C.choose("fwd", (256, 56, 56, 64), w, (1, 1), (0, 0, 0, 0), (1, 1))
    b = C.choose("fwd", (64, 56, 56, 64), w, (1, 1), (0, 0, 0, 0), (1, 1))
    assert a == b


def test_flat_space_padded_rows_stay_zero():
    """A variable with ``pad_rows`` gets zero rows after it in master, gradient and shadow (the tied BERT decoder's
    30720-row vocabulary): the padded views alias the variable, the fused updates keep the pad at zero, and the
    layout of every other variable is unchanged apart from the offset."""
    from mdtf.ops import optim
    from mdtf.parallel.flat import FlatParamSpace
    torch.manual_seed(0)
    a = V.Variable("emb", torch.randn(10, 4))
    b = V.Variable("bias", torch.randn(10))
    c = V.Variable("other", torch.randn(3, 4))
    a.pad_rows = b.pad_rows = 6
    space = FlatParamSpace([a, b, c], "cpu", torch.bfloat16)
    for v, rows in ((a, 16), (b, 16)):
        assert v.master_padded.shape[0] == rows and v.grad_padded.shape[0] == rows
        assert v.shadow_padded.shape[0] == rows
        assert v.master_padded.data_ptr() == v.master.data_ptr()
        assert v.grad_padded.data_ptr() == v.grad.data_ptr()
        assert v.shadow_padded.data_ptr() == v.shadow.data_ptr()
        assert not v.master_padded[v.shape[0]:].any() and not v.shadow_padded[v.shape[0]:].any()
    assert c.master_padded is None
    a0, c0 = a.master.clone(), c.master.clone()
    for kind in ("momentum", "adam"):
        for g in space.groups:
            g.grad.normal_()
            a.grad_padded[10:].zero_()          # a sum of zero products, as the decoder writes it
            b.grad_padded[10:].zero_()
            if kind == "momentum":
                optim.momentum_(g.master, g.grad, g.state_buffer("m"), g.shadow, 0.1, 0.9, weight_decay=1e-2)
            else:
                optim.adam_(g.master, g.grad, g.state_buffer("m1"), g.state_buffer("v1"), g.shadow, 0.01, 0.9, 0.999,
                            1e-8, 1, weight_decay=1e-2)
        for v in (a, b):
            assert not v.master_padded[v.shape[0]:].any() and not v.shadow_padded[v.shape[0]:].any()
    assert not torch.equal(a.master, a0) and not torch.equal(c.master, c0)
    assert torch.equal(c.shadow, c.master.to(torch.bfloat16))


def test_bert_tied_decoder_padding_on_the_build_pass(tmp_path):
    """BERT reserves the decoder's zero rows on the word embedding and the MLM bias during the build pass, so the
    flat space has the padded views; training keeps the pad at zero and the checkpoint keeps the [vocab, H] shapes."""
    from mdtf.models import Bert, BertPretrainingLoss, SyntheticBertLoader
    from mdtf.ops import nn as ops
    from mdtf.train.saver import Saver
    V.reset_default_graph()
    S.reset()
    P = 4
    ld = SyntheticBertLoader(16, P, vocab=1000, seed=0)
    ld.batch_size = 2
    raw, gt = ld.load_train_batch()
    opt = mdtf.train.AdamWeightDecayOptimizer(1e-3, weight_decay_rate=0.01)
    tg = []
    Tower(Net(Bert("tiny", vocab_size=1000, seq_len=16, max_predictions=P)), "tower_0/", tg, raw, gt,
          BertPretrainingLoss(P), opt, batch_size=2).process()
    op = opt.apply_gradients(Tower.average_gradients(tg), global_step=mdtf.train.get_or_create_global_step())
    sess = mdtf.train.MonitoredTrainingSession(log_step_count_steps=0)
    for _ in range(2):
        sess.run(op)
    pad = ops.decoder_pad_rows(1000)
    store = V.get_store()
    emb = store.vars["bert/embeddings/word_embeddings"]
    bias = store.vars["cls/predictions/output_bias"]
    for v in (emb, bias):
        assert v.pad_rows == pad > 0
        assert v.master_padded.shape[0] == 1000 + pad
        assert not v.master_padded[1000:].any() and not v.grad_padded[1000:].any()
    path = Saver().save(sess, str(tmp_path / "ckpt"))
    from mdtf.ckpt.tensor_bundle import BundleReader
    r = BundleReader(path)
    assert tuple(r.get_tensor("bert/embeddings/word_embeddings").shape) == (1000, 128)
    assert tuple(r.get_tensor("cls/predictions/output_bias").shape) == (1000,)
