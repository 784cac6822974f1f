"""Variables, variable scopes, collections and the global step.

The reference builds a TF1 graph in which ``tf.get_variable`` inside
``tf.variable_scope`` creates (or, with reuse, looks up) named variables
(``distribute_tools.py:24-66``, ``distribute_tower.py:45-48``), losses are
gathered through graph collections (``distribute_tower.py:70-76,131-135``) and
``global_step`` is a non-trainable int64 variable (``distribute_train.py:106``).

Eager re-design: user model code runs every step.  The *first* execution
("build" pass, run once by :class:`~mdtf.runtime.tower.Tower`) creates the
variables; later executions look them up (the store is "frozen").  Variable
names are the scope paths (``conv1/weights``), which are also the checkpoint
tensor names.

Every trainable variable keeps an fp32 master tensor.  When the store has a
reduced compute dtype (bf16 on MI355X), ``get_variable`` hands the model a
bf16 *shadow* that the fused optimizer kernel rewrites after each update
(no per-step cast kernels); the backward of that read accumulates straight
into the variable's slot of the flat gradient buffer and notifies the
gradient reducer, so bucketed RCCL all-reduces start while backward is still
running (see ``mdtf/parallel/reducer.py``).
"""
import collections
import os
import contextlib
import math
import re
import threading

import torch

AUTO_REUSE = "AUTO_REUSE"


class GraphKeys(object):
    GLOBAL_VARIABLES = "variables"
    TRAINABLE_VARIABLES = "trainable_variables"
    LOSSES = "losses"
    SUMMARIES = "summaries"
    UPDATE_OPS = "update_ops"
    MOVING_AVERAGE_VARIABLES = "moving_average_variables"


# ---------------------------------------------------------------------------
# initializers (distribute_tools.py:62,75,100,103,135,200,203,215,223)
# ---------------------------------------------------------------------------
def _fans(shape):
    shape = list(shape)
    if len(shape) < 1:
        return 1, 1
    if len(shape) == 1:
        return shape[0], shape[0]
    if len(shape) == 2:
        return shape[0], shape[1]
    receptive = 1
    for d in shape[:-2]:
        receptive *= d
    return shape[-2] * receptive, shape[-1] * receptive  # HWIO: fan_in = kh*kw*cin


def constant_initializer(value=0.0):
    def init(shape, dtype, generator=None):
        return torch.full(shape, float(value), dtype=dtype)
    return init


zeros_initializer = lambda: constant_initializer(0.0)  # noqa: E731
ones_initializer = lambda: constant_initializer(1.0)   # noqa: E731


def truncated_normal_initializer(mean=0.0, stddev=1.0, dtype=None):
    def init(shape, dtype_, generator=None):
        t = torch.empty(shape, dtype=torch.float32)
        torch.nn.init.trunc_normal_(t, mean=mean, std=stddev, a=mean - 2 * stddev, b=mean + 2 * stddev,
                                    generator=generator)
        return t.to(dtype_)
    return init


def random_normal_initializer(mean=0.0, stddev=1.0):
    def init(shape, dtype, generator=None):
        t = torch.empty(shape, dtype=torch.float32)
        t.normal_(mean, stddev, generator=generator)
        return t.to(dtype)
    return init


def random_uniform_initializer(minval=-0.05, maxval=0.05):
    def init(shape, dtype, generator=None):
        t = torch.empty(shape, dtype=torch.float32)
        t.uniform_(minval, maxval, generator=generator)
        return t.to(dtype)
    return init


def xavier_initializer(uniform=True):
    """Glorot init on TF-layout shapes (HWIO for conv, [in, out] for FC)."""
    def init(shape, dtype, generator=None):
        fan_in, fan_out = _fans(shape)
        t = torch.empty(shape, dtype=torch.float32)
        if uniform:
            lim = math.sqrt(6.0 / (fan_in + fan_out))
            t.uniform_(-lim, lim, generator=generator)
        else:
            std = math.sqrt(2.0 / (fan_in + fan_out))
            torch.nn.init.trunc_normal_(t, std=std, a=-2 * std, b=2 * std, generator=generator)
        return t.to(dtype)
    return init


glorot_uniform_initializer = xavier_initializer


def variance_scaling_initializer(scale=2.0, mode="fan_in"):
    """He init (ResNet)."""
    def init(shape, dtype, generator=None):
        fan_in, fan_out = _fans(shape)
        n = {"fan_in": fan_in, "fan_out": fan_out, "fan_avg": (fan_in + fan_out) / 2.0}[mode]
        std = math.sqrt(scale / max(n, 1))
        t = torch.empty(shape, dtype=torch.float32)
        torch.nn.init.trunc_normal_(t, std=std, a=-2 * std, b=2 * std, generator=generator)
        return t.to(dtype)
    return init


# ---------------------------------------------------------------------------
class Variable(object):
    """A named framework variable: fp32 master + optional compute shadow."""

    def __init__(self, name, tensor, trainable=True, keep_fp32=False, collections_=None):
        self.name = name
        self.master = tensor                # fp32 (or int) leaf tensor
        self.trainable = trainable
        self.keep_fp32 = keep_fp32          # never shadowed to the compute dtype (BN affine, biases of fp32 ops)
        self.shadow = None                  # compute-dtype copy kept in sync by the optimizer
        self.grad = None                    # gradient slot (a view of the flat grad buffer once flattened)
        self.ps_task = None                 # PS shard owning this variable (replica_device_setter)
        self.device_hint = None
        self.index = -1                     # position in the trainable list
        self.on_grad_ready = None           # reducer callback(variable), fired when all uses are back
        self.uses = 0                       # reads under grad mode in the current step
        self.bucket = None
        self.collections = list(collections_ or [])
        self.initial_value = None
        self.apply_weight_decay = tensor.dim() > 1   # optimizer-fused decay: weights yes, biases/BN no
        self.pad_rows = 0                   # zero rows reserved after the variable in the flat buffers
        self.master_padded = self.grad_padded = self.shadow_padded = None   # their views (parallel/flat.py)

    @property
    def shape(self):
        return tuple(self.master.shape)

    @property
    def dtype(self):
        return self.master.dtype

    @property
    def op_name(self):
        return self.name

    def numel(self):
        return self.master.numel()

    def value(self):
        return self.master

    def assign(self, value):
        with torch.no_grad():
            self.master.copy_(torch.as_tensor(value, dtype=self.master.dtype).to(self.master.device))
            if self.shadow is not None:
                self.shadow.copy_(self.master)

    def refresh_shadow(self):
        if self.shadow is not None:
            with torch.no_grad():
                self.shadow.copy_(self.master)

    def read(self, compute_dtype=None):
        """The tensor the model computes with (autograd-connected)."""
        if not self.trainable:
            return self.master                      # moving statistics etc. are updated in place
        if torch.is_grad_enabled():
            self.uses += 1
            out = _VarRead.apply(_grad_token(), self, compute_dtype)
            out._mdtf_var = self          # lets fused kernels accumulate straight into the grad slot
            return out
        if self.shadow is not None:
            return self.shadow
        if compute_dtype is not None and not self.keep_fp32 and self.master.dtype != compute_dtype:
            return self.master.detach().to(compute_dtype)
        return self.master.detach()

    def __repr__(self):
        return "<mdtf.Variable %r shape=%s dtype=%s>" % (self.name, self.shape, self.dtype)


_TOKEN = None


def _grad_token():
    """A 0-d leaf that requires grad: makes autograd call ``_VarRead.backward``
    while the master tensors themselves stay plain (in-place-updatable) views
    of the flat parameter buffer."""
    global _TOKEN
    if _TOKEN is None:
        _TOKEN = torch.zeros((), requires_grad=True)
    return _TOKEN


class _VarRead(torch.autograd.Function):
    """Forward: the shadow (or master); backward: accumulate into the grad slot."""

    @staticmethod
    def forward(ctx, token, var, compute_dtype):
        ctx.var = var
        master = var.master
        if var.shadow is not None:
            return var.shadow.detach()      # fresh alias: autograd metadata never lands on the shadow
        if compute_dtype is not None and not var.keep_fp32 and master.dtype != compute_dtype:
            return master.detach().to(compute_dtype)
        return master.detach()

    @staticmethod
    def backward(ctx, g):
        var = ctx.var
        if var.grad is None:
            var.grad = torch.zeros_like(var.master)
        if not _is_marker(g):             # a sink-only gradient was already accumulated in place
            note_accumulate(var)
            var.grad.add_(g)              # one kernel, dtype promotion included
        grad_done(var)
        return None, None, None


_MARKERS = {}


def grad_marker(t):
    """Zero-cost stand-in gradient for ``t`` (an expanded 1-element zero tensor)."""
    key = (t.dtype, t.device)
    base = _MARKERS.get(key)
    if base is None:
        base = torch.zeros(1, dtype=t.dtype, device=t.device)
        _MARKERS[key] = base
    return base.expand(t.shape)


def _is_marker(g):
    base = _MARKERS.get((g.dtype, g.device))
    return base is not None and g.data_ptr() == base.data_ptr() and all(st == 0 for st in g.stride())


def grad_sink(t):
    """The Variable whose fp32 grad slot a kernel may accumulate into directly.

    Returns the Variable when ``t`` is the value a Variable handed to the model
    (under grad mode) and its grad slot exists, else None.  A backward that
    uses the sink *adds* its gradient into ``var.grad`` (zeroed at the start of
    every step) and returns :func:`grad_marker` as the autograd gradient of
    ``t``; ``_VarRead.backward`` then skips the add (or adds only the other
    consumers' gradients) and fires the bucket hook as usual.  This removes the
    zero/cast/add kernels between a weight-gradient kernel and the flat
    gradient buffer that RCCL reduces.
    """
    var = getattr(t, "_mdtf_var", None)
    if var is None or var.grad is None or var.grad.dtype != torch.float32 or not var.grad.is_contiguous():
        return None
    return var


# Store-first gradient slots (MDTF_GRAD_STORE_FIRST, on by default): a weight-gradient kernel that writes every
# element of a slot and is the step's FIRST writer of it overwrites it instead of accumulating (the other writers
# of the step -- a shared weight's other consumers -- accumulate onto it).  A variable whose first write of a step was such a store is not zeroed at the start of the next
# step (parallel/flat.py skips its range in the one zero-fill launch), which removes its share of the gradient
# buffer fill and the read of C in the kernel's epilogue.  Safety nets: any other first write into a skipped slot
# zeroes it first (note_accumulate, _VarRead.backward), and a skipped slot nobody wrote in a step is zeroed at the
# end of backward (unclaimed_skips).
GRAD_EPOCH = [0]
STORE_FIRST = os.environ.get("MDTF_GRAD_STORE_FIRST", "1") != "0"


def begin_grad_epoch():
    GRAD_EPOCH[0] += 1


def claim_store(var):
    """True when the caller's kernel -- which writes EVERY element of ``var.grad`` -- may overwrite the slot: it is
    the step's first write into it (later writers of the step, e.g. the other consumers of a shared weight,
    accumulate onto it as usual); records the claim."""
    if var is None or getattr(var, "written_epoch", -1) == GRAD_EPOCH[0]:
        return False
    if not STORE_FIRST:
        note_accumulate(var)
        return False
    var.written_epoch = GRAD_EPOCH[0]
    var.store_first = True
    return True


def unclaim_store(var):
    """Undo claim_store() when the kernel did not run: the fallback's accumulation needs a zeroed slot."""
    var.written_epoch = -1
    var.store_first = False
    note_accumulate(var)


def note_accumulate(var):
    """An accumulating write into ``var.grad``: the first one of the step zeroes a slot the fill skipped."""
    if var is None or getattr(var, "written_epoch", -1) == GRAD_EPOCH[0]:
        return
    var.written_epoch = GRAD_EPOCH[0]
    var.store_first = False
    if getattr(var, "skip_zero", False) and var.grad is not None:
        var.grad.zero_()


def unclaimed_skips(variables):
    """Skipped (not zeroed) slots nobody wrote this step: zero them (their gradient is 0) and stop skipping."""
    for v in variables:
        if getattr(v, "skip_zero", False) and getattr(v, "written_epoch", -1) != GRAD_EPOCH[0]:
            v.grad.zero_()
            v.store_first = False


def grad_done(var):
    """One use of ``var`` has contributed its gradient (fires the bucket hook)."""
    var.uses -= 1
    if var.uses <= 0 and var.on_grad_ready is not None:
        var.on_grad_ready(var)


# ---------------------------------------------------------------------------
class _Scope(object):
    def __init__(self, name, reuse):
        self.name = name
        self.reuse = reuse
        self._reuse_set = False

    def reuse_variables(self):
        self.reuse = True


class VariableStore(object):
    """Process-wide registry of named variables + per-step collections."""

    def __init__(self):
        self.vars = collections.OrderedDict()
        self.device = torch.device("cpu")
        self.compute_dtype = None
        self.frozen = False
        self.flat = None                   # FlatParamSpace once built
        self._local = threading.local()
        self._collections = collections.defaultdict(list)
        self._persistent_collections = collections.defaultdict(list)
        self.placement_fn = None           # replica_device_setter policy
        self.generator = torch.Generator().manual_seed(0)
        self.global_step = None

    # -- scope stacks (thread local) ---------------------------------------
    def _stack(self):
        st = getattr(self._local, "scopes", None)
        if st is None:
            st = [_Scope("", False)]
            self._local.scopes = st
        return st

    def _name_stack(self):
        st = getattr(self._local, "names", None)
        if st is None:
            st = []
            self._local.names = st
        return st

    def current_scope(self):
        return self._stack()[-1]

    def scope_name(self):
        return self._stack()[-1].name

    def name_scope_name(self):
        ns = self._name_stack()
        return ns[-1] if ns else ""

    # -- variable creation ---------------------------------------------------
    def get_variable(self, name, shape=None, dtype=torch.float32, initializer=None, trainable=True,
                     collections_=None, keep_fp32=False, reuse=None):
        scope = self.current_scope()
        full = "%s/%s" % (scope.name, name) if scope.name else name
        if reuse is None:
            reuse = scope.reuse
        if full in self.vars:
            if not self.frozen and reuse is False:
                raise ValueError("Variable %s already exists, disallowed. Did you mean to set reuse=True "
                                 "or reuse=AUTO_REUSE in VarScope?" % full)
            v = self.vars[full]
            if shape is not None and tuple(shape) != v.shape:
                raise ValueError("Trying to share variable %s, but specified shape %s and found shape %s." % (
                    full, tuple(shape), v.shape))
            return v.read(self.compute_dtype)
        if reuse is True and not self.frozen:
            raise ValueError("Variable %s does not exist, or was not created with get_variable(). "
                             "Did you mean to set reuse=AUTO_REUSE in VarScope?" % full)
        if self.flat is not None:
            raise RuntimeError("Variable %s created after the parameter space was finalized; create every "
                               "variable during the build pass" % full)
        if shape is None:
            raise ValueError("shape is required to create variable %s" % full)
        if dtype is None:
            dtype = torch.float32
        if initializer is None:
            initializer = xavier_initializer() if torch.empty((), dtype=dtype).is_floating_point() \
                else constant_initializer(0)
        elif not callable(initializer):
            initializer = constant_initializer(initializer)
        t = initializer(tuple(shape), dtype, generator=self.generator)
        t = t.to(self.device)
        v = Variable(full, t, trainable=trainable and t.is_floating_point(), keep_fp32=keep_fp32,
                     collections_=collections_)
        if self.placement_fn is not None:
            self.placement_fn(v)
        if v.trainable:
            v.index = sum(1 for x in self.vars.values() if x.trainable)
        self.vars[full] = v
        for c in (collections_ or []):
            self._persistent_collections[c].append(v)
        return v.read(self.compute_dtype)

    def variable(self, name):
        return self.vars[name]

    def trainable_variables(self):
        return [v for v in self.vars.values() if v.trainable]

    def global_variables(self):
        return list(self.vars.values())

    # -- collections ------------------------------------------------------
    def add_to_collection(self, name, value):
        self._collections[name].append((self.name_scope_name(), value))

    def get_collection(self, name, scope=None):
        if name == GraphKeys.TRAINABLE_VARIABLES:
            items = self.trainable_variables()
            return [v for v in items if scope is None or re.match(scope, v.name)]
        if name == GraphKeys.GLOBAL_VARIABLES:
            items = self.global_variables()
            return [v for v in items if scope is None or re.match(scope, v.name)]
        out = [val for (ns, val) in self._collections.get(name, [])
               if scope is None or ns.startswith(scope.rstrip("/"))]
        out += [v for v in self._persistent_collections.get(name, [])
                if scope is None or re.match(scope, v.name)]
        return out

    def clear_step_collections(self):
        self._collections.clear()

    def reset(self):
        self.__init__()


_STORE = VariableStore()


def get_store():
    return _STORE


def reset_default_graph():
    """Drop every variable/collection (tests; TF's reset_default_graph)."""
    _STORE.reset()


# ---------------------------------------------------------------------------
# TF-style module-level API
# ---------------------------------------------------------------------------
def get_variable(name, shape=None, dtype=torch.float32, initializer=None, trainable=True,
                 collections=None, keep_fp32=False, reuse=None):
    return _STORE.get_variable(name, shape, dtype, initializer, trainable, collections, keep_fp32, reuse)


@contextlib.contextmanager
def variable_scope(name_or_scope, reuse=None, default_name=None):
    stack = _STORE._stack()
    parent = stack[-1]
    if isinstance(name_or_scope, _Scope):
        name = name_or_scope.name
    else:
        nm = name_or_scope if name_or_scope is not None else default_name
        name = ("%s/%s" % (parent.name, nm) if parent.name and nm else (nm or parent.name))
    if reuse is None:
        reuse = parent.reuse
    elif reuse is False and parent.reuse is True:
        reuse = True  # reuse is inherited (TF semantics)
    sc = _Scope(name, reuse)
    stack.append(sc)
    ns = _STORE._name_stack()
    ns.append(name)
    try:
        yield sc
    finally:
        stack.pop()
        ns.pop()


def get_variable_scope():
    return _STORE.current_scope()


def find_variable(name):
    """The :class:`Variable` object ``name`` names in the current scope (None if absent), whatever the grad mode
    (``get_variable`` returns its read, which carries the object only under grad mode)."""
    scope = _STORE.current_scope()
    return _STORE.vars.get("%s/%s" % (scope.name, name) if scope.name else name)


@contextlib.contextmanager
def name_scope(name):
    ns = _STORE._name_stack()
    parent = ns[-1] if ns else ""
    full = "%s/%s" % (parent, name) if parent else name
    ns.append(full)
    try:
        yield full + "/"
    finally:
        ns.pop()


def add_to_collection(name, value):
    _STORE.add_to_collection(name, value)


def get_collection(name, scope=None):
    return _STORE.get_collection(name, scope)


def trainable_variables():
    return _STORE.trainable_variables()


def global_variables():
    return _STORE.global_variables()


@contextlib.contextmanager
def device(spec):
    """``tf.device`` analogue: accepts a device string or a device-setter.

    Process-per-GPU means compute placement is fixed per process; the spec is
    recorded for variable placement bookkeeping (PS shard ownership).
    """
    prev = _STORE.placement_fn
    if callable(spec):
        _STORE.placement_fn = spec
    try:
        yield
    finally:
        _STORE.placement_fn = prev


# ---------------------------------------------------------------------------
class GlobalStep(object):
    """The int64 ``global_step`` variable; a host counter kept in lockstep."""

    name = "global_step"

    def __init__(self, value=0):
        self._value = int(value)

    def value(self):
        return self._value

    def assign(self, v):
        self._value = int(v)

    def increment(self, n=1):
        self._value += n
        return self._value

    def __int__(self):
        return self._value

    def __repr__(self):
        return "<GlobalStep %d>" % self._value


def get_or_create_global_step():
    if _STORE.global_step is None:
        _STORE.global_step = GlobalStep(0)
    return _STORE.global_step


def get_global_step():
    return _STORE.global_step


create_global_step = get_or_create_global_step
