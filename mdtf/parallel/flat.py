"""Flat parameter space: every trainable variable re-homed into a few
contiguous HBM buffers, pre-partitioned into gradient buckets.

Why (MI355X-first): the reference updates each variable separately on PS CPUs
(``distribute_train.py:151-158``) and averages tower gradients per variable
(``distribute_tower.py:78-114``).  With contiguous buffers

* the gradient reduction is a handful of large RCCL collectives over xGMI —
  buckets are contiguous slices, so there are no pack/unpack copies;
* the optimizer is ONE fused kernel launch per group (``mdtf/ops/optim.py``),
  which also refreshes the bf16 compute shadow of the weights.

Variables are grouped by (shadow dtype, weight-decay flag).  Inside a group the
layout is *reverse creation order*, so the tail of the forward pass (the first
gradients of backward) fills the first bucket.  Each bucket is padded to a
multiple of ``pad_to`` (= world size in PS-shard mode) so that
reduce-scatter/all-gather shards are equal and contiguous.

A variable with ``pad_rows > 0`` gets that many zero rows reserved after it in
every buffer (master, gradient, shadow), exposed as ``master_padded`` /
``grad_padded`` / ``shadow_padded`` views of ``rows + pad_rows`` rows: the tied
BERT decoder reads the vocabulary as 30720 rows (a multiple of its split-K
chunks) without a per-step copy.  The pad rows stay exactly zero: their master
starts at zero, their gradient is only ever a sum of zero products, and every
fused update maps (w, g) = (0, 0) to 0.
"""
import collections

import torch

_ALIGN = 64  # elements; 256-B aligned fp32 / 128-B aligned bf16 slices


def _round_up(x, m):
    return -(-x // m) * m


def _extent(v):
    """Elements a variable occupies in the flat buffers, trailing zero rows included."""
    pad = int(getattr(v, "pad_rows", 0) or 0)
    if pad <= 0 or len(v.shape) == 0:
        return v.numel()
    return v.numel() + pad * (v.numel() // max(v.shape[0], 1))


class Bucket(object):
    __slots__ = ("group", "index", "start", "end", "variables", "pending", "work", "launched",
                 "shard_offset", "shard_len", "updated", "gather")

    def __init__(self, group, index, start, end, variables):
        self.group = group
        self.index = index
        self.start = start
        self.end = end
        self.variables = variables
        self.pending = 0
        self.work = None
        self.launched = False
        self.updated = False       # sharded overlap: shard updated + gather issued during backward
        self.gather = None
        self.shard_offset = 0
        self.shard_len = 0

    @property
    def numel(self):
        return self.end - self.start


class FlatGroup(object):
    def __init__(self, variables, device, shadow_dtype, decay, bucket_elems=None, pad_to=1):
        self.variables = list(variables)
        self.device = device
        self.shadow_dtype = shadow_dtype
        self.decay = decay
        self.pad_to = max(int(pad_to), 1)
        bucket_elems = bucket_elems or (1 << 62)
        self.offsets = []
        self.buckets = []
        off = 0
        bstart, bvars = 0, []
        for v in self.variables:
            self.offsets.append(off)
            bvars.append(v)
            off += _round_up(_extent(v), _ALIGN)
            if off - bstart >= bucket_elems:
                off = bstart + _round_up(off - bstart, _ALIGN * self.pad_to)
                self.buckets.append(Bucket(self, len(self.buckets), bstart, off, bvars))
                bstart, bvars = off, []
        if bvars:
            off = bstart + _round_up(off - bstart, _ALIGN * self.pad_to)
            self.buckets.append(Bucket(self, len(self.buckets), bstart, off, bvars))
        self.numel = off
        self.master = torch.zeros(self.numel, dtype=torch.float32, device=device)
        self.grad = torch.zeros(self.numel, dtype=torch.float32, device=device)
        self.shadow = torch.zeros(self.numel, dtype=shadow_dtype, device=device) if shadow_dtype else None
        self.state = {}
        for b in self.buckets:
            for v in b.variables:
                v.bucket = b
        for v, o in zip(self.variables, self.offsets):
            n = v.numel()
            mview = self.master[o:o + n].view(v.shape)
            mview.copy_(v.master.detach().to(device))
            v.master = mview
            v.grad = self.grad[o:o + n].view(v.shape)
            if self.shadow is not None:
                sview = self.shadow[o:o + n].view(v.shape)
                sview.copy_(mview)
                v.shadow = sview
            e = _extent(v)
            if e > n:
                pshape = (v.shape[0] + int(v.pad_rows),) + tuple(v.shape[1:])
                v.master_padded = self.master[o:o + e].view(pshape)
                v.grad_padded = self.grad[o:o + e].view(pshape)
                v.shadow_padded = self.shadow[o:o + e].view(pshape) if self.shadow is not None else None
            v.flat_group = self
            v.flat_offset = o

    def state_buffer(self, name, numel=None):
        key = (name, numel or self.numel)
        if key not in self.state:
            self.state[key] = torch.zeros(numel or self.numel, dtype=torch.float32, device=self.device)
        return self.state[key]

    def zero_grad(self, skip_stored=False):
        """Zero the gradient buffer.  ``skip_stored``: leave out the slots whose first write of the previous step
        was a store (``variables.claim_store``; this step's writer overwrites them again) -- one fill launch over
        the remaining ranges."""
        skips = []
        for v in self.variables:
            v.skip_zero = bool(skip_stored and getattr(v, "store_first", False))
            if v.skip_zero:
                skips.append((v.flat_offset, v.numel()))
        if len(skips) > 1000:       # more holes than the one-launch fill takes (kFillMaxRanges): zero everything
            for v in self.variables:
                v.skip_zero = False
            skips = []
        if not skips:
            self.grad.zero_()
            return
        key = tuple(skips)
        cached = getattr(self, "_fill_ranges", None)
        if cached is None or cached[0] != key:
            ranges, pos = [], 0
            for o, n in sorted(skips):
                if o > pos:
                    ranges.append((pos, o - pos))
                pos = max(pos, o + n)
            if pos < self.numel:
                ranges.append((pos, self.numel - pos))
            total = sum(n for _, n in ranges)
            rt = torch.tensor([x for r in ranges for x in r], dtype=torch.int64).to(self.grad.device)
            cached = self._fill_ranges = (key, ranges, rt, total)
        _, ranges, rt, total = cached
        if self.grad.is_cuda and ranges:
            from ..ops import _native as N
            if "mdtf_fill_ranges_zero" not in N.SIGNATURES:
                N.register("mdtf_fill_ranges_zero", [N.P, N.P, N.I, N.L, N.P])
            N.check(N.fn("mdtf_fill_ranges_zero")(N.ptr(self.grad), N.ptr(rt), len(ranges), total,
                                                   N.stream_ptr(self.grad.device)), "fill_ranges_zero")
        else:
            for o, n in ranges:
                self.grad[o:o + n].zero_()

    def refresh_shadow(self):
        if self.shadow is not None:
            self.shadow.copy_(self.master)


class FlatParamSpace(object):
    """All trainable variables of the store, flattened into groups."""

    def __init__(self, variables, device, compute_dtype=None, bucket_bytes=None, pad_to=1):
        self.device = device
        self.compute_dtype = compute_dtype
        bucket_elems = (bucket_bytes // 4) if bucket_bytes else None
        by_key = collections.OrderedDict()
        for v in reversed(list(variables)):
            shadow = compute_dtype if (compute_dtype is not None and not v.keep_fp32
                                       and compute_dtype != torch.float32) else None
            by_key.setdefault((shadow, bool(v.apply_weight_decay)), []).append(v)
        self.groups = [FlatGroup(vs, device, sd, dec, bucket_elems, pad_to) for (sd, dec), vs in by_key.items()]
        self.variables = list(variables)

    @property
    def buckets(self):
        return [b for g in self.groups for b in g.buckets]

    def zero_grad(self, skip_stored=False):
        for g in self.groups:
            g.zero_grad(skip_stored)

    def refresh_shadows(self):
        for g in self.groups:
            g.refresh_shadow()

    def numel(self):
        return sum(g.numel for g in self.groups)
