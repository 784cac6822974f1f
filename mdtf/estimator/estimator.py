"""A working ``Estimator`` on the mdtf engine (model_fn / input_fn API).

Reference: ``distribute_estimator.py:14-35`` subclasses ``tf.estimator.Estimator``
and never runs (it imports a missing symbol).  Here the
estimator is real and sits on the same runtime as ``Train``:

* ``model_fn(features, labels, mode[, params][, config]) -> EstimatorSpec`` is
  recorded as a :class:`~mdtf.train.step.TowerProgram` and re-executed
  eagerly each step; ``optimizer.minimize(loss)`` called *inside* model_fn is
  captured (it returns a placeholder op) and turned into one fused
  :class:`~mdtf.train.step.TrainOp` (flat fp32 master/grad buffers, bucketed
  RCCL gradient reduction when a process group is up, one fused optimizer
  launch per group);
* ``train`` runs a ``MonitoredTrainingSession`` on ``model_dir`` (chief
  restore, checkpoint/summary/step-counter hooks from the ``RunConfig``) until
  ``steps``/``max_steps`` or the input is exhausted;
* ``evaluate`` restores the latest checkpoint and averages the loss and the
  ``eval_metric_ops`` over the eval input; ``predict`` yields predictions.

``input_fn()`` may return a ``(features, labels)`` pair of tensors (the same
batch every step), an iterator/generator of such pairs (``StopIteration``
ends the loop, like ``OutOfRangeError``), or a Dataloader whose
``load_train_batch()``/``load_eval_batch()`` handles are used directly.
"""
import collections
import contextlib
import inspect
import os
import tempfile
import threading

import torch

from ..train import hooks as H
from ..train import saver as SV
from ..train import session as SE
from ..train import step as S
from ..train import variables as V
from ..utils import log as logger
from .run_config import RunConfig


class ModeKeys(object):
    TRAIN = "train"
    EVAL = "eval"
    PREDICT = "infer"


class EstimatorSpec(collections.namedtuple("EstimatorSpec", [
        "mode", "predictions", "loss", "train_op", "eval_metric_ops", "training_hooks", "evaluation_hooks",
        "prediction_hooks"])):
    def __new__(cls, mode, predictions=None, loss=None, train_op=None, eval_metric_ops=None, training_hooks=None,
                evaluation_hooks=None, prediction_hooks=None):
        if mode == ModeKeys.TRAIN and (loss is None or train_op is None):
            raise ValueError("EstimatorSpec in TRAIN mode needs loss and train_op")
        if mode == ModeKeys.EVAL and loss is None:
            raise ValueError("EstimatorSpec in EVAL mode needs loss")
        if mode == ModeKeys.PREDICT and predictions is None:
            raise ValueError("EstimatorSpec in PREDICT mode needs predictions")
        return super(EstimatorSpec, cls).__new__(cls, mode, predictions, loss, train_op, dict(eval_metric_ops or {}),
                                                 tuple(training_hooks or ()), tuple(evaluation_hooks or ()),
                                                 tuple(prediction_hooks or ()))


# ------------------------------------------------------------------ capture
_cap = threading.local()


class MinimizeRequest(object):
    """What ``optimizer.minimize(loss)`` returns inside a model_fn (becomes the TrainOp)."""

    def __init__(self, optimizer, global_step, var_list):
        self.optimizer = optimizer
        self.global_step = global_step
        self.var_list = var_list


class _Capture(object):
    def __init__(self):
        self.request = None
        self.spec = None

    @contextlib.contextmanager
    def active(self):
        prev = getattr(_cap, "current", None)
        _cap.current = self
        try:
            yield self
        finally:
            _cap.current = prev

    def record(self, optimizer, global_step, var_list):
        if self.request is None:
            self.request = MinimizeRequest(optimizer, global_step, var_list)
        return self.request


def current_capture():
    return getattr(_cap, "current", None)


# ------------------------------------------------------------------ metrics
class metrics(object):
    """Streaming metrics for ``eval_metric_ops``: each returns ``(batch_value, weight)``."""

    @staticmethod
    def accuracy(labels, predictions):
        labels = labels.reshape(-1).to(predictions.device)
        pred = predictions.reshape(-1)
        return (pred == labels).float().mean(), labels.numel()

    @staticmethod
    def mean(values):
        return values.float().mean(), values.numel()

    @staticmethod
    def mean_squared_error(labels, predictions):
        d = predictions.float() - labels.float().to(predictions.device)
        return (d * d).mean(), d.numel()


# ------------------------------------------------------------------ input
def _to_dev(x, dev):
    if isinstance(x, torch.Tensor):
        return x.to(dev, non_blocking=True)
    if isinstance(x, dict):
        return {k: _to_dev(v, dev) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_dev(v, dev) for v in x)
    return x


class _PairOut(S.SourceOutput):
    """features (index 0) or labels (index 1) of the per-step input pair; dicts allowed."""

    def evaluate(self, ctx):
        key = ("src", id(self.source))
        if key not in ctx.cache:
            ctx.cache[key] = _to_dev(self.source.dequeue(), V.get_store().device)
        return ctx.cache[key][self.index]

    def peek(self):
        return _to_dev(self.source.peek(), V.get_store().device)[self.index]


def _first_tensor(x):
    if isinstance(x, torch.Tensor):
        return x
    if isinstance(x, dict):
        x = list(x.values())
    if isinstance(x, (list, tuple)):
        for v in x:
            t = _first_tensor(v)
            if t is not None:
                return t
    return None


def _input_handles(input_fn, params, mode):
    """(features_handle, labels_handle, batch_size) for an input_fn."""
    sig = inspect.signature(input_fn).parameters if callable(input_fn) else {}
    r = input_fn(params=params) if "params" in sig else input_fn()
    if hasattr(r, "load_train_batch"):               # an mdtf Dataloader
        f, l = r.load_eval_batch() if mode != ModeKeys.TRAIN else r.load_train_batch()
        return f, l, getattr(r, "batch_size", 1)
    if isinstance(r, tuple) and len(r) == 2 and not inspect.isgenerator(r):
        pair = r
        src = S.BatchSource(lambda: pair, name="input_fn")
    elif isinstance(r, (torch.Tensor, dict)):
        pair = (r, None)
        src = S.BatchSource(lambda: pair, name="input_fn")
    else:
        it = iter(r)

        def nxt():
            v = next(it)
            return v if isinstance(v, tuple) and len(v) == 2 else (v, None)
        src = S.BatchSource(nxt, name="input_fn")
    t = _first_tensor(src.peek()[0])
    return _PairOut(src, 0), _PairOut(src, 1), (t.shape[0] if t is not None and t.dim() > 0 else 1)


def _default_device():
    return torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")


class Estimator(object):
    def __init__(self, model_fn, model_dir=None, config=None, params=None, warm_start_from=None):
        if not callable(model_fn):
            raise TypeError("model_fn must be callable")
        self._model_fn = model_fn
        config = config or RunConfig()
        if model_dir is None:
            model_dir = config.model_dir or tempfile.mkdtemp(prefix="mdtf_estimator_")
            logger.warn("Using temporary folder as model directory: %s" % model_dir)
        if config.model_dir is not None and config.model_dir != model_dir:
            raise ValueError("model_dir %r differs from RunConfig.model_dir %r" % (model_dir, config.model_dir))
        self._config = config.replace(model_dir=model_dir)
        self._model_dir = model_dir
        self._params = dict(params or {})
        self._warm_start_from = warm_start_from
        os.makedirs(model_dir, exist_ok=True)

    model_dir = property(lambda s: s._model_dir)
    config = property(lambda s: s._config)
    params = property(lambda s: dict(s._params))

    def _model_fn_for(self, mode):
        return self._model_fn

    def _call_model_fn(self, fn, features, labels, mode):
        sig = inspect.signature(fn).parameters
        kw = {}
        if "mode" in sig:
            kw["mode"] = mode
        if "params" in sig:
            kw["params"] = self._params
        if "config" in sig:
            kw["config"] = self._config
        spec = fn(features, labels, **kw) if "labels" in sig else fn(features, **kw)
        if not isinstance(spec, EstimatorSpec):
            raise ValueError("model_fn must return an EstimatorSpec, got %r" % type(spec))
        return spec

    def _build(self, input_fn, mode):
        V.reset_default_graph()
        S.reset()
        store = V.get_store()
        store.device = _default_device()
        store.compute_dtype = torch.bfloat16 if store.device.type == "cuda" else None
        if self._config.tf_random_seed is not None:
            store.generator.manual_seed(int(self._config.tf_random_seed))
        feats, labels, bs = _input_handles(input_fn, self._params, mode)
        cap = _Capture()
        fn = self._model_fn_for(mode)

        def program(f, l):
            with cap.active():
                spec = self._call_model_fn(fn, f, l, mode)
            cap.spec = spec
            out = {}
            if spec.loss is not None:
                out["loss"] = spec.loss
            if spec.predictions is not None:
                out["predictions"] = spec.predictions
            if spec.eval_metric_ops:
                out["metrics"] = spec.eval_metric_ops
            return out
        prog = S.TowerProgram(program, (feats, labels), name="estimator")
        with S.training_mode(mode == ModeKeys.TRAIN):
            prog.build(bs)
        V.get_store().frozen = True
        gs = V.get_or_create_global_step()
        return prog, cap, gs

    # ---------------------------------------------------------------- train
    def latest_checkpoint(self):
        return SV.latest_checkpoint(self._model_dir)

    def get_variable_names(self):
        from ..ckpt import tensor_bundle
        ckpt = self.latest_checkpoint()
        if ckpt is None:
            raise ValueError("no checkpoint in %s" % self._model_dir)
        return sorted(tensor_bundle.BundleReader(ckpt).keys())

    def get_variable_value(self, name):
        from ..ckpt import tensor_bundle
        return tensor_bundle.BundleReader(self.latest_checkpoint()).get_tensor(name)

    def train(self, input_fn, hooks=None, steps=None, max_steps=None, saving_listeners=None):
        if steps is not None and max_steps is not None:
            raise ValueError("Can not provide both steps and max_steps.")
        if max_steps is not None:
            ckpt = self.latest_checkpoint()
            if ckpt is not None and _step_of(ckpt) >= max_steps:
                logger.info("Skipping training since max_steps has already saved.")
                return self
        prog, cap, gs = self._build(input_fn, ModeKeys.TRAIN)
        req = cap.request
        if req is None:
            raise ValueError("model_fn in TRAIN mode must build train_op with optimizer.minimize(loss, ...)")
        loss_h = prog.output("loss")
        train_op = req.optimizer.minimize(loss_h, global_step=gs, var_list=req.var_list)
        all_hooks = list(hooks or []) + list(cap.spec.training_hooks)
        if steps is not None or max_steps is not None:
            all_hooks.append(H.StopAtStepHook(num_steps=steps, last_step=max_steps))
        cfg = self._config
        scaffold = SE.Scaffold(init_fn=self._warm_start_fn())
        ckpt_hooks = list(saving_listeners or [])
        sess = SE.MonitoredTrainingSession(
            is_chief=cfg.is_chief, checkpoint_dir=self._model_dir, scaffold=scaffold, hooks=all_hooks,
            save_checkpoint_secs=cfg.save_checkpoints_secs, save_checkpoint_steps=cfg.save_checkpoints_steps,
            save_summaries_steps=cfg.save_summary_steps, log_step_count_steps=cfg.log_step_count_steps)
        for h in sess._hooks:
            if isinstance(h, H.CheckpointSaverHook):
                for lst in ckpt_hooks:
                    h._listeners.append(lst)
        self.last_loss = None
        try:
            while not sess.should_stop():
                try:
                    _, lv = sess.run([train_op, loss_h])
                except StopIteration:
                    break
                self.last_loss = float(lv)
        finally:
            sess.close()
        return self

    def _warm_start_fn(self):
        ws = self._warm_start_from
        if ws is None:
            return None

        def init_fn(scaffold, session):
            path = ws if not os.path.isdir(ws) else SV.latest_checkpoint(ws)
            SV.Saver(save_optimizer_state=False).restore(session, path)
            logger.info("Warm-started from %s" % path)
        return init_fn

    # ---------------------------------------------------------------- eval
    def _restore(self, checkpoint_path):
        ckpt = checkpoint_path or self.latest_checkpoint()
        if ckpt is None:
            raise ValueError("Could not find trained model in model_dir: %s." % self._model_dir)
        SV.Saver(save_optimizer_state=False).restore(None, ckpt)
        return ckpt

    def evaluate(self, input_fn, steps=None, hooks=None, checkpoint_path=None, name=None):
        prog, cap, gs = self._build(input_fn, ModeKeys.EVAL)
        ckpt = self._restore(checkpoint_path)
        total_loss, n = 0.0, 0
        sums, weights = collections.defaultdict(float), collections.defaultdict(float)
        while steps is None or n < steps:
            ctx = S.RunContext()
            try:
                out = prog.forward(ctx, grad=False)
            except StopIteration:
                break
            total_loss += float(out["loss"])
            for k, v in (out.get("metrics") or {}).items():
                val, w = (v if isinstance(v, tuple) else (v, 1.0))
                sums[k] += float(val) * float(w)
                weights[k] += float(w)
            n += 1
            if isinstance(prog.inputs[0], _PairOut) and steps is None and _is_constant(prog.inputs[0]):
                break
        res = {"loss": total_loss / max(n, 1), "global_step": V.get_global_step().value()}
        for k in sums:
            res[k] = sums[k] / max(weights[k], 1e-12)
        logger.info("Saving dict for global step %d: %s" % (res["global_step"], ", ".join(
            "%s = %g" % (k, v) for k, v in sorted(res.items()))))
        out_dir = os.path.join(self._model_dir, "eval" if not name else "eval_" + name)
        os.makedirs(out_dir, exist_ok=True)
        import json
        with open(os.path.join(out_dir, "results.json"), "a") as f:
            f.write(json.dumps(dict(res, checkpoint=os.path.basename(ckpt))) + "\n")
        return res

    def predict(self, input_fn, predict_keys=None, hooks=None, checkpoint_path=None, yield_single_examples=True):
        prog, cap, gs = self._build(input_fn, ModeKeys.PREDICT)
        self._restore(checkpoint_path)
        constant = _is_constant(prog.inputs[0])
        while True:
            ctx = S.RunContext()
            try:
                out = prog.forward(ctx, grad=False)
            except StopIteration:
                return
            preds = out["predictions"]
            if isinstance(preds, dict) and predict_keys:
                preds = {k: preds[k] for k in predict_keys}
            preds = _to_dev(preds, torch.device("cpu"))
            if yield_single_examples:
                n = _first_tensor(preds).shape[0]
                for i in range(n):
                    yield {k: v[i] for k, v in preds.items()} if isinstance(preds, dict) else preds[i]
            else:
                yield preds
            if constant:
                return


def _is_constant(pair_out):
    fn = getattr(pair_out.source, "_fn", None)
    return fn is not None and fn.__name__ == "<lambda>"


def _step_of(ckpt):
    try:
        return int(ckpt.rsplit("-", 1)[1])
    except (IndexError, ValueError):
        return 0
