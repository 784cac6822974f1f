"""Deferred "graph" handles on an eager backend.

The reference builds a TF1 graph once and then calls
``sess.run([train_op, global_step, loss], feed_dict=...)`` in its hot loop
(``distribute_train.py:183-193``).  To keep that run loop source-compatible
on eager PyTorch, graph-building calls return lightweight *handles*:

* :class:`Placeholder` — resolved from ``feed_dict``;
* :class:`SourceOutput` — one element of a batch dequeued once per ``run``;
* :class:`StepTensor` — an output (``loss``, ``logits``...) of a recorded
  :class:`TowerProgram` (the closure ``Tower.process`` records);
* :class:`TrainOp` — one fused training step: forward/backward of every
  tower program, bucketed gradient reduction over RCCL overlapped with
  backward, one fused optimizer launch per parameter group, global-step
  increment.

A ``Session.run`` evaluates the TrainOp first, so ``loss`` fetched beside it
is the loss of that training step — exactly the TF semantics of fetching both
from one graph execution.  Fetching a StepTensor without a TrainOp runs the
program forward-only in inference mode (used by ``Eval``).
"""
import contextlib
import itertools
import threading

import torch

from . import variables as V

_state = threading.local()


def is_training():
    return getattr(_state, "training", True)


@contextlib.contextmanager
def training_mode(flag):
    prev = is_training()
    _state.training = bool(flag)
    try:
        yield
    finally:
        _state.training = prev


class Fetchable(object):
    _mdtf_fetch = True

    def evaluate(self, ctx):
        raise NotImplementedError


class RunContext(object):
    _ids = itertools.count(1)

    def __init__(self, feed_dict=None, session=None):
        self.id = next(self._ids)
        self.feed_dict = feed_dict or {}
        self.session = session
        self.cache = {}
        self.stop_requested = False

    def request_stop(self):
        self.stop_requested = True


def _to_device(t, device):
    if isinstance(t, torch.Tensor):
        return t.to(device, non_blocking=True) if t.device != device else t
    return t


class Placeholder(Fetchable):
    def __init__(self, dtype=torch.float32, shape=None, name=None):
        self.dtype = dtype
        self.shape = shape
        self.name = name or "Placeholder"

    def evaluate(self, ctx):
        if self not in ctx.feed_dict:
            raise KeyError("You must feed a value for placeholder %s" % self.name)
        v = ctx.feed_dict[self]
        if not isinstance(v, torch.Tensor):
            import numpy as np
            v = torch.as_tensor(np.asarray(v))
        if self.dtype is not None and v.dtype != self.dtype and v.is_floating_point():
            v = v.to(self.dtype)
        return _to_device(v, V.get_store().device)

    def dummy(self, batch_size):
        shape = [batch_size if (s is None or s == -1) else s for s in (self.shape or [batch_size])]
        return torch.zeros(shape, dtype=self.dtype or torch.float32, device=V.get_store().device)


def placeholder(dtype=torch.float32, shape=None, name=None):
    return Placeholder(dtype, shape, name)


class BatchSource(object):
    """A per-step batch producer (``dequeue()`` returns a tuple of tensors)."""

    def __init__(self, fn, name="batch"):
        self._fn = fn
        self.name = name
        self._peeked = None

    def peek(self):
        if self._peeked is None:
            self._peeked = self._fn()
        return self._peeked

    def dequeue(self):
        if self._peeked is not None:
            b, self._peeked = self._peeked, None
            return b
        return self._fn()

    def outputs(self, n):
        return tuple(SourceOutput(self, i) for i in range(n))


class SourceOutput(Fetchable):
    def __init__(self, source, index):
        self.source = source
        self.index = index

    def evaluate(self, ctx):
        key = ("src", id(self.source))
        if key not in ctx.cache:
            batch = self.source.dequeue()
            ctx.cache[key] = tuple(_to_device(b, V.get_store().device) for b in batch)
        return ctx.cache[key][self.index]

    def peek(self):
        return _to_device(self.source.peek()[self.index], V.get_store().device)


def resolve(x, ctx):
    if isinstance(x, Fetchable):
        return x.evaluate(ctx)
    if isinstance(x, (list, tuple)):
        return type(x)([resolve(i, ctx) for i in x])
    if isinstance(x, dict):
        return {k: resolve(v, ctx) for k, v in x.items()}
    return x


def build_value(x, batch_size):
    """Concrete stand-in values for the variable-building pass."""
    if isinstance(x, Placeholder):
        return x.dummy(batch_size)
    if isinstance(x, SourceOutput):
        return x.peek()
    if isinstance(x, (list, tuple)):
        return type(x)(build_value(i, batch_size) for i in x)
    if isinstance(x, dict):
        return {k: build_value(v, batch_size) for k, v in x.items()}
    return x


class TowerProgram(object):
    """A recorded per-replica computation ``fn(*resolved_inputs) -> dict``."""

    def __init__(self, fn, inputs, name="tower_0"):
        self.fn = fn
        self.inputs = inputs
        self.name = name
        self.last_outputs = None

    def build(self, batch_size=1):
        """Variable-creation pass (TF graph construction)."""
        store = V.get_store()
        with torch.no_grad():
            out = self._call(build_value(self.inputs, batch_size))
        store.clear_step_collections()
        return out

    def _call(self, args):
        store = V.get_store()
        store.clear_step_collections()
        out = self.fn(*args)
        if not isinstance(out, dict):
            out = {"output": out}
        return out

    def forward(self, ctx, grad):
        key = ("prog", id(self))
        if key in ctx.cache:
            return ctx.cache[key]
        args = resolve(self.inputs, ctx)
        with torch.set_grad_enabled(grad), training_mode(grad):
            out = self._call(args)
        ctx.cache[key] = out
        self.last_outputs = out
        return out

    def output(self, key):
        return StepTensor(self, key)


def _host_value(t):
    if isinstance(t, torch.Tensor):
        t = t.detach()
        if t.device.type == "cpu":
            return t.item() if t.dim() == 0 else t.numpy()
        return t
    return t


class StepTensor(Fetchable):
    def __init__(self, program, key):
        self.program = program
        self.key = key
        self.name = "%s/%s" % (program.name, key)

    def evaluate(self, ctx):
        out = ctx.cache.get(("prog", id(self.program)))
        if out is None:
            out = self.program.forward(ctx, grad=False)
        return _host_value(out[self.key])

    def raw(self, ctx):
        return ctx.cache[("prog", id(self.program))][self.key]


class GradRef(Fetchable):
    """``(gradient, variable)`` gradient handle: the variable's flat grad slot."""

    def __init__(self, var, program=None):
        self.var = var
        self.program = program

    def evaluate(self, ctx):
        return _host_value(self.var.grad)


def compute_gradients(loss, var_list=None):
    if not isinstance(loss, StepTensor):
        raise TypeError("compute_gradients expects the loss handle returned by a Tower/TowerProgram")
    store = V.get_store()
    vs = var_list if var_list is not None else store.trainable_variables()
    vs = [store.vars[v] if isinstance(v, str) else v for v in vs]
    return [(GradRef(v, loss.program), v) for v in vs]


class TrainOp(Fetchable):
    """One synchronous training step (see module docstring)."""

    def __init__(self, optimizer, grads_and_vars, global_step=None, sync=False):
        self.optimizer = optimizer
        self.grads_and_vars = list(grads_and_vars)
        self.variables = [v for _, v in self.grads_and_vars]
        progs = []
        for g, _ in self.grads_and_vars:
            p = getattr(g, "program", None)
            if p is not None and p not in progs:
                progs.append(p)
        losses = getattr(grads_and_vars, "loss_handles", None)
        self.programs = progs
        self.loss_key = "loss"
        self.global_step = global_step
        self.sync = sync
        self.reducer = None
        self.space = None
        self.step_count = 0
        self.grad_scale_extra = 1.0 / max(len(self.programs), 1)
        self.last_contributed = True
        self.graph = None
        _register(self)

    # -- finalisation: flat buffers + reducer ----------------------------
    def finalize(self, process_group=None, store=None):
        if self.space is not None:
            return
        from ..parallel.flat import FlatParamSpace
        from ..parallel.reducer import GradReducer
        from ..config import constants
        import torch.distributed as dist
        vstore = V.get_store()
        distributed = dist.is_available() and dist.is_initialized()
        world = dist.get_world_size(process_group) if distributed else 1
        opt = self.optimizer
        mode = getattr(opt, "mode", "allreduce")
        bucket_bytes = getattr(opt, "bucket_bytes", None) or constants.bucket_bytes()
        overlap = getattr(opt, "overlap", True) and len(self.programs) <= 1
        self.space = FlatParamSpace(self.variables, vstore.device, vstore.compute_dtype, bucket_bytes,
                                    pad_to=world if mode == "sharded" else 1)
        vstore.flat = self.space
        vstore.frozen = True
        R = getattr(opt, "replicas_to_aggregate", None)
        if R is not None and distributed:
            # replicas are counted in towers (one per rank)
            pass
        self.reducer = GradReducer(self.space, process_group, mode=mode, overlap=overlap,
                                   replicas_to_aggregate=R, store=store,
                                   comm_dtype=getattr(opt, "comm_dtype", None))

    # -- execution ---------------------------------------------------------
    def _graph_enabled(self):
        from . import graph as G
        flag = getattr(self.optimizer, "hip_graph", None)
        if flag is None:
            flag = G.env_enabled()
            if not flag:
                try:
                    from ..config.flags import FLAGS
                    flag = bool(getattr(FLAGS, "hip_graph", False))
                except Exception:
                    flag = False
        return bool(flag) and torch.cuda.is_available()

    def _run_step(self, ctx, step, dyn=None):
        """forward + backward of every tower program, reduction, fused update (one step)."""
        from ..ops import conv as _conv
        from ..ops import gemm as _gemm
        red = self.reducer
        red.begin_step()
        lr = self.optimizer.learning_rate(step)
        if red.R == red.world:
            # sharded mode: buckets are updated + all-gathered during backward with the (known) 1/N scale
            pre_scale = (1.0 / red.world) * self.grad_scale_extra
            red.set_update_fn(lambda t: self.optimizer.update(t, lr, pre_scale, self.step_count, dyn=dyn))
        else:
            red.set_update_fn(None)
        red.fork_update_stream()               # inside a capture: the side stream of the in-backward updates
        _conv._WT.step_begin()                 # conv filters' K-contiguous copies: one batched refresh per step
        _gemm._CATS.step_begin()               # q|k|v weight concatenations: one batched copy per step
        try:
            for prog in self.programs:
                out = prog.forward(ctx, grad=True)
                loss = out[self.loss_key]
                red.join_zero()                # the side-stream gradient zeroing ran beside the forward
                loss.backward()
        finally:
            _conv._WT.step_end()
            _gemm._CATS.step_end()
        scale = red.end_backward(step) * self.grad_scale_extra
        with torch.no_grad():
            for target in red.update_targets():
                self.optimizer.update(target, lr, scale, self.step_count, dyn=dyn)
            red.after_update()
        return scale

    def release_graph(self):
        """Free the captured step graph (and its private memory pool).  Must run before the
        process group it captured collectives of is destroyed; the next step re-captures."""
        if self.graph is not None:
            self.graph.release()
            self.graph = None

    def evaluate(self, ctx):
        key = ("train", id(self))
        if key in ctx.cache:
            return None
        if self.space is None:
            self.finalize()
        step = self.global_step.value() if self.global_step is not None else self.step_count
        if self.graph is None and self._graph_enabled():
            from .graph import StepGraph
            self.graph = StepGraph(self)
        if self.graph is not None:
            self.graph.run(ctx, step)
        else:
            self._run_step(ctx, step)
        if STEP_FAULTS:
            # fault injection inside the step, after its collectives and update (mdtf.cluster.health
            # FaultInjectionHook mode "abort_in_step"): a one-shot callable that raises
            STEP_FAULTS.pop(0)(step)
        c = self.reducer.contributed
        # (a device 0/1 mask for GPU backup workers: a per-step snapshot of the persistent mask buffer, which
        # the next step / graph replay rewrites in place; converted lazily by whoever reads it)
        if isinstance(c, torch.Tensor):
            c = c.clone()
        self.last_contributed = c
        self.step_count += 1
        if self.global_step is not None:
            self.global_step.increment()
        ctx.cache[key] = True
        return None


_TRAIN_OPS = []
STEP_FAULTS = []        # one-shot callables(step) raised from inside TrainOp.evaluate (fault injection)


def _register(op):
    _TRAIN_OPS.append(op)


def train_ops():
    return list(_TRAIN_OPS)


def release_graphs():
    for op in _TRAIN_OPS:
        op.release_graph()
    from ..ops import conv as _conv
    from ..ops import gemm as _gemm
    _conv._WT.clear()               # the filter-transpose cache holds the released space's shadows
    _gemm._CATS.clear()


def reset():
    release_graphs()
    del _TRAIN_OPS[:]
