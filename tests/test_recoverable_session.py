"""In-process session recovery (TF's _RecoverableSession under MonitoredTrainingSession; reference
distribute_train.py:169-180): an AbortedError / UnavailableError during run() re-creates the session
from the latest checkpoint and training continues to the same final state as an uninterrupted run."""
import os
import sys

import pytest
import torch

sys.path.insert(0, os.path.dirname(__file__))


def _train(md, last_step, fault_at=None, mode="abort", max_recoveries=None, save_steps=2):
    import dist_helpers
    import mdtf
    from mdtf.cluster.health import FaultInjectionHook
    from mdtf.train import hooks as H
    from mdtf.train import step as S
    from mdtf.train import variables as V
    V.reset_default_graph()
    S.reset()
    Lin, MSE, xs, ys, x_ph, y_ph, Tower, Net = dist_helpers._linear_setup(0, 1, 4)
    opt = mdtf.train.MomentumOptimizer(0.1, 0.9)
    tg = []
    Tower(Net(Lin()), "tower_0/", tg, x_ph, y_ph, MSE(), opt, batch_size=4).process()
    gs = mdtf.train.get_or_create_global_step()
    op = opt.apply_gradients(Tower.average_gradients(tg), global_step=gs)
    hooks = [H.StopAtStepHook(last_step=last_step)]
    if fault_at is not None:
        hooks.append(FaultInjectionHook("worker", 0, step=fault_at, task="worker:0", mode=mode))
    g = torch.Generator().manual_seed(7)
    data = [(torch.randn(4, 8, generator=g), torch.randn(4, 1, generator=g)) for _ in range(last_step + 1)]
    with mdtf.train.MonitoredTrainingSession(checkpoint_dir=md, save_checkpoint_steps=save_steps, hooks=hooks,
                                             log_step_count_steps=0, max_recoveries=max_recoveries) as sess:
        while not sess.should_stop():
            xb, yb = data[gs.value()]                   # the batch is a function of the global step
            sess.run(op, feed_dict={x_ph: xb, y_ph: yb})
        rec = sess.recoveries
    return gs.value(), {v.name: v.master.detach().clone() for v in V.get_store().trainable_variables()}, rec


@pytest.mark.parametrize("mode", ["abort", "unavailable"])
def test_recovers_from_checkpoint_and_matches_uninterrupted(mode, tmp_path):
    step_ref, w_ref, _ = _train(str(tmp_path / "ref"), 8)
    step, w, rec = _train(str(tmp_path / "run"), 8, fault_at=5, mode=mode)
    assert rec == 1 and step == step_ref == 8
    for k in w_ref:
        assert torch.allclose(w[k], w_ref[k], atol=1e-6), k


def test_recovery_budget_exhausted_raises(tmp_path):
    from mdtf import errors
    with pytest.raises(errors.AbortedError):
        _train(str(tmp_path / "run"), 8, fault_at=3, max_recoveries=0)


def test_store_failures_map_to_unavailable():
    from mdtf import errors

    class DistStoreError(RuntimeError):
        pass
    e = errors.as_recoverable(DistStoreError("connection reset"))
    assert isinstance(e, errors.UnavailableError)
    assert errors.as_recoverable(ValueError("bug")) is None
    assert isinstance(errors.as_recoverable(errors.AbortedError(message="x")), errors.AbortedError)
