"""Fan-out activation gradients accumulated in place (no autograd add kernel).

A ResNet block input feeds two consumers: the first conv of the block and
the residual branch (the identity into the last BatchNorm, or the projection
conv).  In stock autograd each consumer returns its own full-size gradient and
the engine adds them (a read-read-write bf16 pass per block).  Here the
producing BatchNorm attaches an :class:`ActGradSink` to its output.  A
sink-aware consumer writes its gradient straight into the sink buffer:
- the first contributor's tensor is adopted as the buffer;
- a later contributor accumulates into it (the v2 conv dgrad epilogue and the
  BN backward's residual-gradient store both have an accumulate mode);
- the contributor then returns ``None`` to autograd.
The producer's backward (called with ``None`` once all consumers are done)
takes the summed gradient from the sink. It also adds whatever ordinary autograd
gradient arrived, so consumers that are not sink-aware stay correct.

A strided 1x1 projection conv may leave its data gradient *deferred* (``pconv``: the gradient, filter, stride and
a closure that runs it): when the contributor that completes the sum is the block's 1x1 / stride-1 conv on the
weight-stationary kernel, both data gradients run as one GEMM (``mdtf_conv_ws_dual``) and the block input's
gradient is written once; anything else runs the closure first.

A ReLU'd residual BatchNorm's backward may leave its contribution *pending* instead of writing it:
``(g, mask)`` meaning ``g * mask`` (the identity shortcut's gradient).  A conv dgrad that supports a
masked accumulate source (:meth:`target_ex`) folds it into its own epilogue, so that tensor is never
written and re-read; any other access materialises it first (``mdtf_mask_mul``).
"""
import os

import torch



class ActGradSink(object):
    """``consumers``: sink-aware consumers registered in the forward.  ``stat_req``: what the
    producing BatchNorm needs for its backward statistics, ``(x, relu_mask[, early_finalize])``.  The contributor that
    completes the sum (the ``consumers``-th) may emit the statistics in its epilogue into ``stats``
    (the v2 conv dgrad does)."""
    __slots__ = ("buf", "count", "consumers", "stat_req", "stats", "pend", "pconv", "early")

    def __init__(self):
        self.buf = None
        self.count = 0
        self.consumers = 0
        self.stat_req = None
        self.stats = None
        self.pend = None
        self.pconv = None
        self.early = None       # (workspace, done event) of a backward finalize issued early (ops.bn)

    def idle(self):
        """Nothing contributed yet (neither written nor left pending / deferred)."""
        return self.buf is None and self.pend is None and self.pconv is None

    def defer_conv(self, dy, w, stride, run):
        """Contribute a strided 1x1 conv's data gradient without running it (only as the first contribution);
        ``run(out, accumulate)`` computes it the ordinary way and returns the tensor written."""
        assert self.idle()
        self.pconv = (dy, w, stride, run)
        self.count += 1

    def take_conv(self):
        """The deferred conv contribution ``(dy, w, stride)`` for a kernel that fuses it (cleared), or None."""
        if self.pconv is None or self.buf is not None or self.pend is not None:
            return None
        dy, w, stride, _ = self.pconv
        self.pconv = None
        return dy, w, stride

    def defer_masked(self, g, mask):
        """Contribute ``g * mask`` without materialising it (only as the first contribution)."""
        assert self.buf is None and self.pend is None
        self.pend = (g, mask)
        self.count += 1

    def _materialize(self):
        if self.pconv is not None:
            run, self.pconv = self.pconv[3], None
            self.buf = run(self.buf, self.buf is not None)
        if self.pend is None:
            return
        from . import _native as N
        g, mask = self.pend
        self.pend = None
        acc = self.buf is not None
        out = self.buf if acc else torch.empty_like(g)
        N.check(N.fn("mdtf_mask_mul")(N.ptr(g), N.ptr(mask), N.ptr(out), g.numel(), int(acc), N.stream_ptr()),
                "mask_mul")
        self.buf = out

    def target_ex(self):
        """(buffer, accumulate, pending) for a kernel that can also fold a pending ``(g, mask)`` into its
        epilogue: with ``pending`` not None, write ``result + g * mask`` into ``buffer`` (None: allocate)."""
        if self.pend is not None and self.buf is None and self.pconv is None:
            p, self.pend = self.pend, None
            FOLDED[0] += 1
            return None, False, p
        self._materialize()
        return self.buf, self.buf is not None, None

    def register(self):
        self.consumers += 1
        return self

    def completing(self):
        """True when the next contribution completes the gradient (every registered consumer)."""
        return self.count + 1 == self.consumers

    def adopt_or_add(self, g):
        """Contribute a materialised gradient tensor."""
        self._materialize()
        if self.buf is None:
            self.buf = g
        else:
            self.buf.add_(g)
        self.count += 1

    def target(self):
        """(buffer, accumulate) for a kernel that writes its contribution in place; call
        :meth:`written` after launching it.  ``None`` buffer: allocate and write (accumulate False)."""
        self._materialize()
        return self.buf, self.buf is not None

    def written(self, buf):
        self.buf = buf
        self.count += 1

    def take(self, dy):
        """Producer side: the total gradient (autograd's ``dy`` may be None)."""
        if self.count == 0:
            return dy
        self._materialize()
        total = self.buf
        if dy is not None:
            total = total.add_(dy)
        self.buf, self.count = None, 0
        return total

    def take_stats(self):
        """The emitted BN statistics ``(psum, psq, slots)`` or None (cleared)."""
        st, self.stats = self.stats, None
        return st

    def take_early(self):
        """The early backward finalize ``(ws, event)`` or None (cleared)."""
        e, self.early = self.early, None
        return e


ENABLED = os.environ.get("MDTF_ACT_SINKS", "1") != "0"      # switch for A/B tests and benches
FOLDED = [0]         # pending masked contributions folded into a dgrad epilogue (tests)
# residual BN backward leaves the identity shortcut's gradient pending (MDTF_MASKED_RESIDUAL=0: written)
MASKED_RESIDUAL = os.environ.get("MDTF_MASKED_RESIDUAL", "1") != "0"


def attach(t):
    if not ENABLED:
        return None
    s = ActGradSink()
    try:
        t._mdtf_act_sink = s
    except AttributeError:          # pragma: no cover
        return None
    return s


def sink_of(t):
    return getattr(t, "_mdtf_act_sink", None) if t is not None else None
