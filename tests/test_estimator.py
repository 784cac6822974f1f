"""Estimator / DistributeEstimator / DistributeExperiment / RunConfig (CPU)."""
import json
import os

import pytest
import torch

import mdtf
from mdtf.estimator import (DistributeEstimator, DistributeExperiment, Estimator, EstimatorSpec, ModeKeys,
                            RunConfig, current_input, metrics)


def _data(n=256, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, 8, generator=g)
    w = torch.randn(8, 3, generator=g)
    y = (x @ w).argmax(1)
    return x, y


def model_fn(features, labels, mode, params):
    h = mdtf.layers.tools.FC_layer("fc1", features, 32) if hasattr(mdtf, "layers") else None
    with mdtf.variable_scope("out"):
        w = mdtf.get_variable("weights", [32, 3], initializer=mdtf.train.variables.xavier_initializer())
        b = mdtf.get_variable("biases", [3], initializer=mdtf.train.variables.constant_initializer(0.0))
    logits = mdtf.nn.matmul(h, w) + b
    preds = logits.argmax(-1)
    if mode == ModeKeys.PREDICT:
        return EstimatorSpec(mode, predictions={"classes": preds, "logits": logits})
    loss = mdtf.nn.sparse_softmax_cross_entropy_with_logits(labels, logits).mean()
    if mode == ModeKeys.EVAL:
        return EstimatorSpec(mode, loss=loss, eval_metric_ops={"accuracy": metrics.accuracy(labels, preds)})
    opt = mdtf.train.AdamOptimizer(params.get("lr", 1e-2))
    train_op = opt.minimize(loss, global_step=mdtf.train.get_global_step())
    return EstimatorSpec(mode, loss=loss, train_op=train_op)


def _batches(x, y, bs=32, epochs=1):
    def input_fn():
        for _ in range(epochs):
            for i in range(0, x.shape[0], bs):
                yield x[i:i + bs], y[i:i + bs]
    return input_fn


def test_estimator_train_eval_predict_resume(tmp_path):
    import mdtf.layers  # noqa: F401
    x, y = _data()
    cfg = RunConfig(save_checkpoints_steps=5, log_step_count_steps=0, tf_random_seed=1)
    est = Estimator(model_fn, model_dir=str(tmp_path), config=cfg, params={"lr": 2e-2})
    est.train(_batches(x, y, epochs=3))                    # until the iterator ends: 3 * 8 steps
    assert est.latest_checkpoint().endswith("-24")
    first = est.last_loss
    r = est.evaluate(_batches(x, y))
    assert r["global_step"] == 24 and r["accuracy"] > 0.6 and r["loss"] < 1.0
    assert os.path.exists(os.path.join(str(tmp_path), "eval", "results.json"))
    # resume: continues from the checkpoint up to max_steps
    est.train(_batches(x, y, epochs=10), max_steps=30)
    assert est.latest_checkpoint().endswith("-30")
    # max_steps already reached -> no-op
    est.train(_batches(x, y), max_steps=30)
    assert est.latest_checkpoint().endswith("-30")
    preds = list(est.predict(_batches(x[:40], y[:40])))
    assert len(preds) == 40 and set(preds[0]) == {"classes", "logits"}
    assert "out/weights" in est.get_variable_names()
    assert est.get_variable_value("out/weights").shape == (32, 3)
    assert first is not None


def test_estimator_constant_input_and_steps(tmp_path):
    import mdtf.layers  # noqa: F401
    x, y = _data(64)
    est = Estimator(model_fn, model_dir=str(tmp_path), config=RunConfig(log_step_count_steps=0),
                    params={"lr": 1e-2})
    est.train(lambda: (x, y), steps=7)
    assert est.latest_checkpoint().endswith("-7")
    est.train(lambda: (x, y), steps=3)
    assert est.latest_checkpoint().endswith("-10")
    r = est.evaluate(lambda: (x, y))
    assert r["global_step"] == 10


def test_estimator_requires_minimize(tmp_path):
    import mdtf.layers  # noqa: F401

    def bad_fn(features, labels, mode):
        with pytest.raises(ValueError):
            EstimatorSpec(mode, loss=None, train_op=None)
        raise RuntimeError("stop")
    x, y = _data(32)
    with pytest.raises(RuntimeError):
        Estimator(bad_fn, model_dir=str(tmp_path)).train(lambda: (x, y), steps=1)


def test_run_config_uid_and_tf_config(monkeypatch):
    a = RunConfig(model_dir="/tmp/a", save_summary_steps=10)
    b = RunConfig(model_dir="/tmp/a", save_summary_steps=99)
    assert a.uid() == b.uid()                       # whitelisted field differs
    c = RunConfig(model_dir="/tmp/b")
    assert a.uid() != c.uid()
    assert "0x" not in a.uid()                      # no object addresses
    monkeypatch.setenv("TF_CONFIG", json.dumps({"cluster": {"ps": ["127.0.0.1:1"], "worker": ["127.0.0.1:2",
                                                                                               "127.0.0.1:3"]},
                                                "task": {"type": "worker", "index": 1}}))
    r = RunConfig()
    assert r.num_ps_replicas == 1 and r.num_worker_replicas == 2 and r.task_id == 1 and not r.is_chief
    assert r.replace(save_checkpoints_steps=3).save_checkpoints_secs is None
    with pytest.raises(ValueError):
        r.replace(nonsense=1)


@current_input(input="SyntheticDataLoader")
class _MyEstimator(DistributeEstimator):
    pass


def test_distribute_estimator_input_annotation(tmp_path):
    est = _MyEstimator(model_fn, model_dir=str(tmp_path))
    from mdtf.data.loaders import SyntheticDataLoader
    assert est.input_class is SyntheticDataLoader
    with pytest.raises(ValueError):
        DistributeEstimator(model_fn, model_dir=str(tmp_path))


def test_distribute_experiment(monkeypatch):
    calls = []
    mdtf.FLAGS.data_load_option = "placeholder"
    try:
        exp = DistributeExperiment("Train", train_fn=lambda dl, mode, pre, post: calls.append(("t", dl, mode)),
                                   train_dataloader="DL")
        exp.run()
        assert calls == [("t", "DL", mdtf.data.loaders.InputOptions.PLACEHOLDER)]
        exp = DistributeExperiment("Eval", eval_fn=lambda dl, pre, post: calls.append(("e", dl)),
                                   eval_dataloader="EDL")
        exp.run()
        assert calls[-1] == ("e", "EDL")
        with pytest.raises(ValueError):
            DistributeExperiment("Train", eval_fn=lambda *a: None)
        with pytest.raises(ValueError):
            DistributeExperiment("Bogus", train_fn=lambda *a: None, train_dataloader="x")
        mdtf.FLAGS.data_load_option = "nonsense"
        with pytest.raises(ValueError):
            DistributeExperiment("Train", train_fn=lambda *a: None, train_dataloader="x")
    finally:
        mdtf.FLAGS.data_load_option = "tfrecords"
