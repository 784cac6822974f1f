"""hipGraph capture of a whole synchronous training step.

The reference builds a TF1 graph once and replays it with
``sess.run([train_op, global_step, loss])`` (``distribute_train.py:183-193``);
TF's executor, not Python, issues the kernels.  mdtf runs eagerly, so a
ResNet-50 step costs ~470 kernel launches from Python (autograd + ctypes):
enough host time that the GPU idles between launches at the start of
backward.  On MI355X the right tool is a HIP graph, not a tracing compiler:
the step — forward, autograd backward, the bucketed RCCL reductions fired from
the gradient hooks, the fused optimizer launches and the PS-shard all-gathers
— is captured once into a ``torch.cuda.CUDAGraph`` (a hipGraph on ROCm) and
replayed as a single launch per step.

Protocol (:class:`StepGraph`, driven by :class:`mdtf.train.step.TrainOp`):

1. ``warmup`` eager steps: conv autotune lookups, lazily created optimizer
   state, RCCL communicator setup, allocator warm-up all happen outside
   capture.
2. Capture: the step's inputs are bound to *static* device buffers, the
   per-step hyper-parameters (LR schedule, Adam bias correction, gradient
   scale) are read by the optimizer kernels from a device buffer ``dyn``
   (``csrc/optim.hip``), so the captured kernel arguments never go stale.
3. Replay: copy the new batch into the static buffers (skipped when the
   loader hands out the same device tensors, e.g. synthetic data), refresh
   ``dyn`` if a value changed, ``graph.replay()``.

A step falls back to eager execution when it cannot be replayed exactly: a
changed input shape or a non-CUDA device.  Backup workers
(``replicas_to_aggregate < N``) are captured too: their contributor mask is
decided on the device (``mdtf.parallel.reducer``, ``csrc/backup.hip``).  Dropout kernels read a
device step counter (:func:`rng_offset_tensor`) so replayed masks differ step
to step.

Enable with ``MDTF_HIP_GRAPH=1``, ``--hip_graph`` (FLAGS) or
``SyncReplicasOptimizer(..., hip_graph=True)``.
"""
import os
import time

import torch

_RNG = {}
LAST_DRAIN = [None]     # how the last capture drained the RCCL watchdog: "recorder" | "refused" (tests)
LAST_DRAIN_POLLS = [0]  # recorder polls the last drain needed before every eager work had retired (tests)


def env_enabled():
    return os.environ.get("MDTF_HIP_GRAPH", "0") not in ("0", "", "false", "False")


def rng_offset_tensor(device):
    """Device int64 step counter mixed into dropout seeds (incremented once per captured step)."""
    key = str(device)
    t = _RNG.get(key)
    if t is None:
        t = torch.zeros(1, dtype=torch.int64, device=device)
        _RNG[key] = t
    return t


_CAPTURED_IDS = set()   # flight-recorder ids of collectives recorded inside a capture (never retired)


def _recorder_entries():
    """Every flight-recorder entry of the process groups (retired ones included), or None when the
    recorder is unavailable or disabled (``TORCH_FR_BUFFER_SIZE`` 0)."""
    try:
        import json
        from torch._C._distributed_c10d import _dump_nccl_trace_json
        d = json.loads(_dump_nccl_trace_json(includeCollectives=True, onlyActive=False))
    except (ImportError, RuntimeError, ValueError, TypeError):
        return None
    ents = d.get("entries")
    if ents is None or (ents and "retired" not in ents[0]):
        return None
    return ents


def _unretired(ents, watermark):
    """Entries issued eagerly before the drain (record id <= watermark) the watchdog still holds."""
    return [e for e in ents if e.get("record_id", -1) <= watermark and e.get("record_id") not in _CAPTURED_IDS
            and not e.get("retired", False)]


def _drain_comm_watchdog(timeout_s=60.0):
    """Wait, on the flight recorder's ``retired`` state and not on a clock, until the RCCL watchdog has
    dropped every eager work.  Returns the record-id watermark (None: not an RCCL job).

    A ProcessGroupNCCL watchdog thread polls the end event of each work issued OUTSIDE capture until it
    retires it; works issued during capture are never handed to it.  A watchdog event query that lands
    while this thread captures raced the capture (the intermittent abort of the RCCL capture test).  The
    dump's ``time_discovered_completed`` (what ``onlyActive`` filters on) is set by the dump itself, so
    "no active entries" says nothing about the watchdog; ``retired`` is set only when the watchdog removed
    the work from its list.  Entries recorded by an earlier capture never retire and are excluded.
    Without a recorder there is no state to wait on: refuse to capture (the caller stays eager)."""
    try:
        import torch.distributed as dist
        if not (dist.is_available() and dist.is_initialized() and dist.get_backend() == "nccl"):
            return None
    except (RuntimeError, ValueError):
        return None
    torch.cuda.synchronize()
    ents = _recorder_entries()
    if ents is None:
        LAST_DRAIN[0] = "refused"
        raise RuntimeError("RCCL flight recorder unavailable (TORCH_FR_BUFFER_SIZE=0?): cannot prove the "
                           "watchdog idle, refusing to capture collectives")
    watermark = max([e.get("record_id", -1) for e in ents] or [-1])
    LAST_DRAIN[0] = "recorder"
    deadline = time.time() + timeout_s
    polls = 0
    while _unretired(ents, watermark):
        if time.time() > deadline:
            raise RuntimeError("RCCL watchdog still holds %d works after %.0f s; refusing to capture"
                               % (len(_unretired(ents, watermark)), timeout_s))
        os.sched_yield()
        polls += 1
        ents = _recorder_entries() or []
    LAST_DRAIN_POLLS[0] = polls
    return watermark


def _note_captured(watermark):
    """Remember the ids the capture recorded: they never retire, later drains skip them."""
    if watermark is None:
        return
    ents = _recorder_entries() or []
    _CAPTURED_IDS.update(e["record_id"] for e in ents if e.get("record_id", -1) > watermark)


def _leaves(x, out):
    from .step import Placeholder, SourceOutput
    if isinstance(x, (Placeholder, SourceOutput)):
        out.append(x)
    elif isinstance(x, (list, tuple)):
        for i in x:
            _leaves(i, out)
    elif isinstance(x, dict):
        for i in x.values():
            _leaves(i, out)
    return out


class _ClonedOutputs(dict):
    """Program outputs of a replayed step: the graph's static tensors are cloned on first
    access, so a fetched ``loss`` keeps its value after the next replay overwrites them."""

    def __init__(self, static):
        super(_ClonedOutputs, self).__init__()
        self._static = static

    def __getitem__(self, k):
        if not dict.__contains__(self, k):
            v = self._static[k]
            dict.__setitem__(self, k, v.detach().clone() if isinstance(v, torch.Tensor) else v)
        return dict.__getitem__(self, k)

    def __contains__(self, k):
        return k in self._static

    def get(self, k, default=None):
        return self[k] if k in self._static else default

    def keys(self):
        return self._static.keys()


class StepGraph(object):
    def __init__(self, op, warmup=2):
        self.op = op
        self.warmup = max(int(warmup), 1)
        self.graph = None
        self.eager_steps = 0
        self.replays = 0
        self.fallbacks = 0
        self.disabled = False       # capture failed once: eager from then on
        self.dyn = None
        self._dyn_vals = None
        self._static_src = {}       # id(source) -> (source, tuple of static tensors)
        self._static_ph = {}        # placeholder -> static tensor
        self._seen_ptrs = {}        # id(source) -> data_ptr tuple per warm-up step
        self._outputs = {}          # id(program) -> static output dict
        self._gs = None

    def release(self):
        """Drop the captured graph, its static buffers and outputs (synchronizes the device)."""
        if self.graph is not None:
            torch.cuda.synchronize()
            self.graph.reset()
            self.graph = None
        self._static_src.clear()
        self._static_ph.clear()
        self._outputs.clear()
        self.dyn = None
        self.eager_steps = 0

    # ------------------------------------------------------------------
    def _inputs(self):
        leaves = []
        for p in self.op.programs:
            _leaves(p.inputs, leaves)
        return leaves

    def _resolve_inputs(self, ctx):
        """Dequeue this step's inputs into ``ctx`` (the same objects the eager path would use)."""
        from .step import SourceOutput
        vals = {}
        for leaf in self._inputs():
            v = leaf.evaluate(ctx)
            if isinstance(leaf, SourceOutput):
                vals[id(leaf.source)] = (leaf.source, ctx.cache[("src", id(leaf.source))])
            else:
                vals[leaf] = v
        return vals

    def _eligible(self):
        red = self.op.reducer
        dev = self.op.space.groups[0].device if self.op.space.groups else None
        if red.world > 1:
            import torch.distributed as dist
            if dist.is_initialized() and dist.get_backend() != "nccl":
                return False            # gloo collectives synchronise with the host: not capturable
        # backup workers qualify when the contributor mask is decided on the device (reducer.backup_device)
        return dev is not None and dev.type == "cuda" and (red.R == red.world or red.backup_device)

    # ------------------------------------------------------------------
    def run(self, ctx, step):
        """Run one training step (eager, capture or replay); returns the gradient scale."""
        if not self._eligible():
            return self.op._run_step(ctx, step)
        if self.disabled:
            return self.op._run_step(ctx, step)
        if self.graph is None:
            if self.eager_steps < self.warmup:
                self.eager_steps += 1
                vals = self._resolve_inputs(ctx)
                self._note_ptrs(vals)
                return self.op._run_step(ctx, step)
            try:
                return self._capture(ctx, step)
            except RuntimeError as e:
                # a capture the runtime rejects (e.g. a collective it cannot record) fails identically on every
                # replica before anything was executed: stay eager for the rest of the run instead of aborting
                from ..utils import log
                log.warn("hipGraph capture failed (%s); running the step eagerly from now on"
                         % (str(e).splitlines() or [""])[0][:200])
                self.disabled = True
                self.graph = None
                torch.cuda.synchronize()
                return self.op._run_step(ctx, step)
        vals = self._resolve_inputs(ctx)
        if not self._bind(vals):
            self.fallbacks += 1
            return self.op._run_step(ctx, step)
        self._set_dyn(step)
        if self.op.reducer.backup_device:
            self.op.reducer.refresh_backup_clock(step)      # host-side, between replays (offsets updated in place)
        self.graph.replay()
        self.replays += 1
        for p in self.op.programs:
            out = _ClonedOutputs(self._outputs[id(p)])
            ctx.cache[("prog", id(p))] = out
            p.last_outputs = out
        return self._gs

    def _note_ptrs(self, vals):
        for k, v in vals.items():
            if isinstance(k, int):
                self._seen_ptrs.setdefault(k, []).append(tuple(t.data_ptr() if isinstance(t, torch.Tensor) else 0
                                                              for t in v[1]))

    def _persistent(self, key, tensors):
        """The loader hands out the same device tensors every step (synthetic data)."""
        seen = self._seen_ptrs.get(key, [])
        now = tuple(t.data_ptr() if isinstance(t, torch.Tensor) else 0 for t in tensors)
        return len(seen) >= 1 and all(s == now for s in seen)

    def _bind(self, vals):
        """Copy this step's inputs into the static buffers; False if a shape changed."""
        copies = []
        for k, v in vals.items():
            if isinstance(k, int):
                static = self._static_src[k][1]
                for t, s in zip(v[1], static):
                    if not isinstance(t, torch.Tensor):
                        continue
                    if t.shape != s.shape or t.dtype != s.dtype:
                        return False
                    if t.data_ptr() != s.data_ptr():
                        copies.append((s, t))
            else:
                s = self._static_ph[k]
                if v.shape != s.shape:
                    return False
                copies.append((s, v))
        for s, t in copies:
            s.copy_(t, non_blocking=True)
        return True

    def _set_dyn(self, step):
        op = self.op
        lr = op.optimizer.learning_rate(step)
        vals = (float(lr), float(op.optimizer.step_size(lr, op.step_count)), float(self._gs))
        if vals != self._dyn_vals:
            host = torch.tensor(vals, dtype=torch.float32).pin_memory()
            self.dyn.copy_(host, non_blocking=True)
            self._dyn_vals = vals

    def _capture(self, ctx, step):
        from .step import RunContext
        op = self.op
        dev = op.space.groups[0].device
        vals = self._resolve_inputs(ctx)
        feed = {}
        cache = {}
        for k, v in vals.items():
            if isinstance(k, int):
                src, tensors = v
                if self._persistent(k, tensors):
                    static = tensors
                else:
                    static = tuple(t.clone() if isinstance(t, torch.Tensor) else t for t in tensors)
                self._static_src[k] = (src, static)
                cache[("src", k)] = static
            else:
                s = v.clone()
                self._static_ph[k] = s
                feed[k] = s
        # the scale is fixed for a replayable step (all replicas contribute)
        red = op.reducer
        self._gs = (1.0 / red.R) * op.grad_scale_extra       # R contributors (= N without backup workers)
        self.dyn = torch.zeros(3, dtype=torch.float32, device=dev)
        self._dyn_vals = None
        self._set_dyn(step)
        rng = rng_offset_tensor(dev)
        fd = dict(ctx.feed_dict)
        fd.update(feed)
        cap_ctx = RunContext(feed_dict=fd, session=ctx.session)
        cap_ctx.cache.update(cache)
        torch.cuda.synchronize(dev)
        watermark = _drain_comm_watchdog()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            rng.add_(1)
            op._run_step(cap_ctx, step, dyn=self.dyn)
        _note_captured(watermark)
        self.graph = g
        for p in op.programs:
            self._outputs[id(p)] = cap_ctx.cache[("prog", id(p))]
        # capture records without executing: run this step now
        g.replay()
        self.replays += 1
        for p in op.programs:
            out = _ClonedOutputs(self._outputs[id(p)])
            ctx.cache[("prog", id(p))] = out
            p.last_outputs = out
        return self._gs
