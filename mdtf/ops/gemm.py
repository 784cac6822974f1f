"""Dense / matmul on the GPU: hand-written MFMA kernels where they win, hipBLASLt GEMMs elsewhere,
fp32 weight-gradient sinks.

Forward: ``y = act(x @ W + b)`` in ONE hand-written MFMA launch (``hand_fwd``: the fd v2 kernel's MODE 3
reads W in place through transposed LDS fragment reads, adds the bias to the fp32 accumulators and applies
GELU/ReLU in the epilogue, also storing the pre-activation GELU's backward needs).  Several weight matrices
that share an input (BERT's query/key/value) are column segments of the same launch, with no concatenated
copy.  Shapes it does not take (and ``MDTF_DENSE_FWD=hipblaslt``) use ``addmm`` (hipBLASLt, bias epilogue)
plus the mdtf activation kernel.

Backward: ``dx = dpre @ W^T`` (bf16; hipBLASLt, or with ``MDTF_DENSE_DGRAD=mdtf`` the mdtf v2 dgrad kernel
for the shapes of ``DGRAD_TILES``; accumulated inside the GEMM into a fanned-out input's gradient sink), and the weight gradient is the mdtf weight-gradient
kernel (``csrc/conv_igemm.hip`` conv_wgrad_v2 run as a 1x1 convolution) writing
*directly into the variable's fp32 gradient slot*.  The same kernel adds the bias
gradient (the column sums of ``dpre``) from the B fragments it already holds, with an
all-ones MFMA, so no bf16 weight gradient is materialised and no column-sum kernel runs.
Shapes the kernel does not take fall back to hipBLASLt ``C += A^T B`` (bf16 inputs, fp32
output) and the two-stage column-sum kernel.
"""
import os

import torch

from . import _native as N
from . import kernels
from . import mm
from . import tunable
from ..train import variables as V

# MDTF_DENSE: "pp" (default) = every dense GEMM the ping-pong MFMA core takes (csrc/gemm_pp.hip: forward with
# bias/activation epilogue, data gradient with the producer's activation backward, weight gradient + bias
# gradient straight into the fp32 slots; q|k|v as segments of one launch); "legacy" = the r2 mix of hipBLASLt
# and the conv-kernel dense paths below (A/B comparisons).
DENSE = os.environ.get("MDTF_DENSE", "pp")
PP = DENSE == "pp"
# Per-product engine inside "pp" (measured on MI355X, profiles/gemm_core_r3.md): the core takes the products where
# it wins end to end -- a forward with a fused activation or several weight segments (no bias_act pass, no
# q|k|v concatenation), and a data gradient that fuses the producer's activation backward or reads segments;
# the plain products stay on hipBLASLt.  Weight gradients (MDTF_PP_WGRAD=wg, default): the split-K weight-gradient
# kernel (csrc/gemm_wg.hip, q|k|v in one launch) where _wg_ok says it wins, else the conv-kernel wgrad; "none" =
# the conv-kernel wgrad everywhere.  MDTF_PP_{FWD,DGRAD,WGRAD} = all | fused | none (FWD also: act = only the forwards
# with a fused activation; the layer's other products then run on the legacy path).  In-step BERT-base kernel
# totals (profiles/bert_engine_ab_r3.md): the core's q|k|v forward (128x192 tiles) and segment dgrad lose to
# hipBLASLt + cat, the GELU-consumer dgrad loses to the conv-kernel fused act dgrad; FFN-in + GELU is a tie
# that saves the bias_act pass.
PP_FWD = os.environ.get("MDTF_PP_FWD", "act")
PP_DGRAD = os.environ.get("MDTF_PP_DGRAD", "fused")
# Per-shape routing on top of the policy above: "KxN,KxN" (K = reduction, N = all output columns of the product) of
# the plain forwards / data gradients that also run on the core.  In-step A/B per product (BERT-base, profiles/ab_r6.md):
# the square 768 x 768 attention-output forward and data gradient are a tie with hipBLASLt (-0.2 % / +0.1 %), so they
# run on the core by default; the K = 3072 products lose on it (FFN-out forward -2.0 %, FFN-in data gradient -1.5 %).
PP_FWD_SHAPES = {s for s in os.environ.get("MDTF_PP_FWD_SHAPES", "768x768").split(",") if s}
PP_DGRAD_SHAPES = {s for s in os.environ.get("MDTF_PP_DGRAD_SHAPES", "768x768").split(",") if s}
PP_WGRAD = os.environ.get("MDTF_PP_WGRAD", "wg")


# MDTF_DENSE_WGRAD_STREAM=1: a dense layer's weight (+ bias) gradients run on the side stream beside the data-gradient
# chain (ops.conv's side stream, joined by the reducer before a bucket is reduced and at the end of backward), so
# the GEMM tails of the two chains overlap; only when every output of the section lands in a gradient slot.
DENSE_WGRAD_STREAM = os.environ.get("MDTF_DENSE_WGRAD_STREAM", "0") == "1"


def _wgrad_section(ctx, x, dpre):
    """Context for a dense backward's weight-gradient section: the side stream when enabled and safe."""
    import contextlib
    sinks = list(ctx.wsinks) + (list(ctx.bsinks) if ctx.has_b else [])
    # every output must be a slot, and this must be each slot's last contribution of the step (uses == 1): an
    # earlier main-stream writer is ordered by the wait below, a later one would race the side stream
    if not (DENSE_WGRAD_STREAM and x.is_cuda and all(sk is not None and getattr(sk, "uses", 1) == 1 for sk in sinks)):
        return contextlib.nullcontext()
    from . import conv as _conv
    side = _conv._side_stream(x.device)
    side.wait_stream(torch.cuda.current_stream(x.device))
    x.record_stream(side)
    dpre.record_stream(side)
    _conv._PENDING.add(x.device)
    return torch.cuda.stream(side)


def _dgrad_shape_on(ws):
    """MDTF_PP_DGRAD_SHAPES names this layer's data-gradient product as "<reduction>x<output columns>" (for a layer
    W [K, N]: "NxK"), the same convention as the forward keys."""
    return bool(PP_DGRAD_SHAPES) and "%dx%d" % (sum(w.shape[1] for w in ws), ws[0].shape[0]) in PP_DGRAD_SHAPES


def _wg_backward(ctx, x, dpre):
    """Weight (+ bias) gradients of a dense layer on the weight-gradient kernel: every segment (q|k|v) in one
    launch straight into the fp32 slots, bias column sums fused (not in deterministic mode: the per-split sums
    are atomics; a column-sum pass then).  False (nothing done) where the kernel does not apply."""
    if PP_WGRAD != "wg" or ctx.trans or any(sk is None for sk in ctx.wsinks):
        return False
    if ctx.has_b and any(sk is None for sk in ctx.bsinks):
        return False
    if not (x.dim() == 2 and x.dtype == torch.bfloat16 and dpre.dtype == torch.bfloat16 and _wg_ok(x, dpre)):
        return False
    fuse_b = ctx.has_b and not N.deterministic()
    # a slot this launch is the step's only writer of is overwritten (V.claim_store: no zero fill, no C read)
    store = [V.claim_store(sk) for sk in ctx.wsinks]
    if not mm.wg_into([sk.grad for sk in ctx.wsinks], x, dpre, dbs=[sk.grad for sk in ctx.bsinks] if fuse_b else None,
                      store=store):
        for sk, st in zip(ctx.wsinks, store):
            if st:                         # not launched: the fallback accumulates into a zeroed slot
                V.unclaim_store(sk)
        return False
    if ctx.has_b and not fuse_b:
        col = 0
        for j, n in enumerate(ctx.widths):
            kernels.colsum_into(dpre[:, col:col + n].contiguous(), ctx.bsinks[j].grad)
            col += n
    return True


def _wg_ok(x, d):
    """Shapes the weight-gradient kernel (csrc/gemm_wg.hip) takes and wins on: K x N weights of 128-multiples over
    >= 4096 tokens.  Until round 5 the square 768 x 768 stayed on the split conv-kernel weight gradient (10 % faster,
    profiles/gemm_wg_probe_r3a.jsonl); with round 6's write-through slabs and store-first slots the weight-gradient
    kernel wins it in the BERT-base step too (+0.4 %, 9.54 vs 9.58 ms, profiles/ab_r6.md).  MDTF_WG_SQUARE=0: the
    conv-kernel path for K * N <= 768 * 768."""
    T, K = x.shape
    Nn = d.shape[1]
    small_ok = os.environ.get("MDTF_WG_SQUARE", "1") == "1"
    return T >= 4096 and K % 128 == 0 and Nn % 128 == 0 and (K * Nn > 768 * 768 or small_ok) and T % 64 == 0


_ACT = {None: 0, "relu": 1, "gelu": 2}
_fp32_out_ok = None      # does this torch build accept addmm(out_dtype=float32, out=...)?
# bias gradients summed inside the weight-gradient kernel (MDTF_FUSED_BIAS_GRAD=0: separate column sums)
FUSED_BIAS_GRAD = os.environ.get("MDTF_FUSED_BIAS_GRAD", "1") != "0"

N.register("mdtf_gemm_wgrad", [N.P, N.P, N.P, N.L, N.I, N.I, N.I, N.I, N.I, N.I, N.I, N.I, N.P, N.I, N.P, N.P])
N.register("mdtf_gemm_fwd", [N.P, N.P, N.P, N.P, N.P, N.I, N.I, N.P, N.P, N.P, N.I, N.L, N.I, N.I, N.I, N.P])

# forward y = act(x W + b) on the hand-written MFMA kernel (csrc/conv_igemm.hip fd v2 MODE 3: W read in place,
# N-contiguous, by transposed LDS fragment reads; bias on the fp32 accumulators; GELU/ReLU and the saved
# pre-activation in the epilogue; q|k|v as column segments of one launch, no concatenated weight copy).
N.register("mdtf_gemm_dgrad_act", [N.P, N.P, N.P, N.P, N.I, N.L, N.I, N.I, N.I, N.I, N.P])

# ffn(): the second layer's data gradient multiplies by the first layer's activation derivative in its epilogue
# (csrc/conv_igemm.hip mdtf_gemm_dgrad_act, fd v2 MODE 4: the epilogue's pre-activation vectors are loaded before
# the main loop, so their HBM latency hides under it), and no separate activation-backward pass runs.  Graph-timed
# 0.071 vs 0.076 ms (hipBLASLt + act backward) at BERT-base's 8192 x 3072 x 768; BERT-base A/B (30 steps,
# alternating): fused 5668 / 5666 vs separate 5661 / 5648 seq/s.  MDTF_FFN_FUSE=0: the separate pass.
FFN_FUSE = os.environ.get("MDTF_FFN_FUSE", "1") != "0"
# (K, N) of the second layer's W [K][N] -> (bm, bn, stages, ver) of the fused data gradient (output K columns)
# (bench/dgrad_act_probe.py, graph-timed at M 8192: 128 x 256 8-wave, 3 stages)
DGRAD_ACT_TILES = {(3072, 768): (128, 256, 3, 3)}
# MDTF_ACT_DGRAD=core: that data gradient on the GEMM core (csrc/gemm_pp.hip, act-backward epilogue with 16-B
# stores) instead of the conv-kernel MODE 4 (A/B switch)
ACT_DGRAD_CORE = os.environ.get("MDTF_ACT_DGRAD", "conv") == "core"

# MDTF_DENSE_FWD: "auto" (default) = the shapes of FWD_TILES, where the kernel beats hipBLASLt inside the
# captured BERT-base step; "mdtf" = every shape it takes; "hipblaslt" = none (torch.addmm + activation kernel).
# Inside the captured BERT-base step (rocprofv3, batch 64 x 128, us per call mdtf / hipBLASLt): q|k|v 62 / 52,
# FFN-in + GELU 78 / 50 + 23 (bias_act), FFN-out and attention-out ~62 / 41 and 20: so the table is empty and the
# library keeps the forward until the kernel wins (bench/dense_fwd_probe.py times both inside graphs).
FWD_MODE = os.environ.get("MDTF_DENSE_FWD", "auto")
HAND_FWD = FWD_MODE != "hipblaslt"
# (K, segment width, segments) -> (bm, bn, stages, ver) at M >= 2048
FWD_TILES = {}


# MDTF_DENSE_WGRAD=hipblaslt: the library's fp32-output GEMM (C += A^T B) and column sums instead (A/B)
HAND_WGRAD = os.environ.get("MDTF_DENSE_WGRAD", "mdtf") != "hipblaslt"


# (K, N) at M >= 4096 -> (bm, bn, splits, slab reduction) of the 4-wave tiles (the ones that also sum the bias
# gradient); bench/dense_wgrad_sweep.py, graph-timed at M 8192, ms new / old choice: 768 x 3072 0.077 / 0.085,
# 3072 x 768 0.073 / 0.080; M < 4096 (768 x 768 at M 1280): 0.0127 / 0.0208
DENSE_WGRAD_TILES = {(768, 3072): (64, 128, 2, False), (3072, 768): (64, 128, 4, True)}


def _wgrad_tile(M, K, Nn):
    if M < 4096:
        return 64, 128, 2, False
    t = DENSE_WGRAD_TILES.get((K, Nn))
    if t is not None:
        return t
    return 64, 128, (8 if K * Nn <= 768 * 768 else 0), True


def wgrad_into(out, x, d, dbias=None):
    """``out[K][N] += x[M][K]^T d[M][N]`` in fp32 (``d`` may be a column slice).

    The mdtf weight-gradient kernel where it applies (K, N multiples of 64 -- it beats
    the library's fp32-output GEMM on the BERT shapes, bench/gemm_micro.py), else
    hipBLASLt.  Deterministic mode uses the unsplit kernel.  ``dbias`` (fp32 [N]): the
    kernel also adds the column sums of ``d`` (the layer's bias gradient) into it, from the
    B fragments it already holds; returns True when it did (else the caller sums them).
    """
    M, K = x.shape
    Nn = d.shape[1]
    if (HAND_WGRAD and K % 64 == 0 and Nn % 64 == 0 and x.is_contiguous() and d.stride(1) == 1 and out.is_contiguous()
            and x.dtype == torch.bfloat16 and d.dtype == torch.bfloat16 and out.dtype == torch.float32):
        bm, bn, splits, use_slab = _wgrad_tile(M, K, Nn)
        if N.deterministic():
            splits = 1
        from . import conv as C
        slab, cap = C.wgrad_slab(M, K, Nn, bm, bn, 2, splits, x.device, dense=True) if use_slab else (None, 0)
        fuse = dbias is not None and FUSED_BIAS_GRAD and dbias.is_contiguous() and dbias.dtype == torch.float32
        with C.slab_side(slab), C.wgrad_tickets(slab):   # grad slots: the slab reduction may leave the chain
            rc = N.fn("mdtf_gemm_wgrad")(N.ptr(x), N.ptr(d), N.ptr(out), M, K, Nn, d.stride(0), out.stride(0), bm, bn,
                                         2, splits, N.ptr(slab), cap, N.ptr(dbias) if fuse else None, N.stream_ptr())
        if rc == 0:
            return fuse
    _accum_mm(out, x.t(), d)
    return False


# data gradient dx[M][K] = dpre[M][N] W[K][N]^T on the hand-written MFMA kernel (csrc/conv_igemm.hip's v2
# dgrad, a 1x1 convolution over M pixels) where it beats hipBLASLt (bench/gemm_hand_probe.py on MI355X,
# BERT-base shapes, ms mdtf / hipBLASLt): K 768 x N 2304 0.047 / 0.055, 768 x 768 0.027 / 0.033,
# 768 x 3072 0.055 / 0.064, M 1280 768 x 768 0.019 / 0.026; K 3072 x N 768 stays on hipBLASLt (0.064 / 0.053)
DGRAD_TILES = {(768, 2304): (128, 128, 2, 2), (768, 768): (128, 256, 2, 3), (768, 3072): (128, 128, 2, 2),
               (1024, 1024): (128, 256, 2, 3), (1024, 3072): (128, 128, 2, 2), (1024, 4096): (128, 128, 2, 2)}
# In the captured BERT-base step the library GEMMs win end to end (A/B, 30 steps, alternating: hipBLASLt
# 5625 / 5582 seq/s vs hand dgrad 5428 / 5473), so the hand-written path is opt-in: MDTF_DENSE_DGRAD=mdtf
HAND_DGRAD = os.environ.get("MDTF_DENSE_DGRAD", "hipblaslt") == "mdtf"


def _hand_dgrad(dpre, w, out=None, accumulate=False):
    """dx = dpre @ w^T on the v2 dgrad kernel, or None when the shape is not in DGRAD_TILES."""
    M, Nn = dpre.shape
    K = w.shape[0]
    tile = DGRAD_TILES.get((K, Nn)) if HAND_DGRAD else None
    if tile is None or dpre.dtype != torch.bfloat16 or not dpre.is_cuda or not w.is_contiguous():
        return None
    if M < 512:
        tile = (64, 128, 3, 2)
    from . import conv as C
    bm, bn, st, ver = tile
    return C.mdtf_dgrad(dpre.view(1, 1, M, Nn), w.view(1, 1, K, Nn), (1, 1, M, K), (1, 1), (0, 0, 0, 0), (1, 1), bm,
                        bn, ver, st, out=out.view(1, 1, M, K) if out is not None else None,
                        accumulate=accumulate).view(M, K)


def _fwd_tile(M, K, nw, nseg):
    """The tile for this shape, or None when "auto" keeps it on hipBLASLt."""
    t = FWD_TILES.get((K, nw, nseg))
    if t is None and FWD_MODE == "auto":
        return None
    if M < 2048:
        return (64, 128, 3, 2) if nw % 128 == 0 else (64, 64, 2, 2)
    if t is not None and nw % t[1] == 0:
        return t
    return (128, 128 if nw % 128 == 0 else 64, 2, 2)


def hand_fwd(x, ws, b, act, tile=None):
    """(y, pre) = (act(x [W_0|..] + b), pre-activation or None) on the MODE 3 kernel, or None if it does not
    take the operands (then the caller uses hipBLASLt)."""
    if not HAND_FWD or not x.is_cuda or x.dtype != torch.bfloat16 or not x.is_contiguous() or len(ws) > 4:
        return None
    M, K = x.shape
    nw = ws[0].shape[1]
    if K % 64 or nw % 64 or any(w.dtype != torch.bfloat16 or not w.is_contiguous() or tuple(w.shape) != (K, nw)
                                for w in ws):
        return None
    ncol = nw * len(ws)
    if b is not None and (b.dtype != torch.bfloat16 or not b.is_contiguous() or b.numel() != ncol):
        return None
    tile = tile or _fwd_tile(M, K, nw, len(ws))
    if tile is None:
        return None
    bm, bn, st, ver = tile
    y = torch.empty((M, ncol), dtype=x.dtype, device=x.device)
    pre = torch.empty_like(y) if act == 2 else None
    p = [N.ptr(w) for w in ws] + [None] * (4 - len(ws))
    from . import conv as C
    rc = N.fn("mdtf_gemm_fwd")(N.ptr(x), p[0], p[1], p[2], p[3], len(ws), nw, N.ptr(b), N.ptr(y), N.ptr(pre), act,
                               M, K, C._v2_code(bm, st, ver), bn, N.stream_ptr())
    if rc != 0:
        return None
    return y, pre


def hand_dgrad_act(dpre, w, pre, act, tile=None):
    """dx = (dpre @ w^T) * act'(pre) on the v2 dgrad kernel with the activation-backward epilogue, or None."""
    if not (dpre.is_cuda and dpre.dtype == torch.bfloat16 and dpre.is_contiguous() and w.is_contiguous()
            and pre.is_contiguous() and w.dtype == torch.bfloat16 and pre.dtype == torch.bfloat16):
        return None
    M, Nn = dpre.shape
    K = w.shape[0]
    if Nn % 64 or K % 8 or tuple(pre.shape) != (M, K) or act not in (1, 2):
        return None
    bm, bn, st, ver = tile or DGRAD_ACT_TILES.get((K, Nn)) or ((128, 128, 2, 2) if M >= 2048 else (64, 128, 3, 2))
    dx = torch.empty((M, K), dtype=dpre.dtype, device=dpre.device)
    from . import conv as C
    rc = N.fn("mdtf_gemm_dgrad_act")(N.ptr(dpre), N.ptr(w), N.ptr(dx), N.ptr(pre), act, M, K, Nn,
                                     C._v2_code(bm, st, ver), bn, N.stream_ptr())
    return dx if rc == 0 else None


class _ActLink(object):
    """Between the two layers of ffn(): the first layer's saved pre-activation (GELU) or output (ReLU), and
    whether the second layer's data gradient already applied the activation derivative."""
    __slots__ = ("pre", "act", "fused")

    def __init__(self):
        self.pre, self.act, self.fused = None, 0, False


def _accum_mm(out, a, b, store=False):
    """``out += a @ b`` (``store``: ``out = a @ b``, out not read) with bf16 a/b and fp32 out."""
    global _fp32_out_ok
    if _fp32_out_ok is None or _fp32_out_ok:
        try:
            torch.addmm(out, a, b, beta=0 if store else 1, out_dtype=torch.float32, out=out)
            _fp32_out_ok = True
            return
        except (RuntimeError, TypeError):
            _fp32_out_ok = False
    if store:
        out.copy_(torch.mm(a, b))
    else:
        out.add_(torch.mm(a, b))


def _act_fwd(pre, act):
    y = torch.empty_like(pre)
    C = pre.shape[-1]
    N.check(N.fn("mdtf_bias_act_fwd")(N.ptr(pre), None, N.ptr(y), None, pre.numel() // C, C, act, N.stream_ptr()),
            "act_fwd")
    return y


def _act_bwd(dy, saved, act):
    dx = torch.empty_like(dy)
    pre = saved if act == 2 else None
    y = saved if act == 1 else None
    N.check(N.fn("mdtf_act_bwd")(N.ptr(dy), N.ptr(pre), N.ptr(y), N.ptr(dx), dy.numel(), act, N.stream_ptr()),
            "act_bwd")
    return dx


def _adjacent(ts):
    """One 1-D view over tensors that lie back to back in memory (e.g. neighbouring slots of the
    flat parameter / gradient buffers), else None."""
    t0 = ts[0]
    if t0 is None or any(t is None or t.dim() != 1 or t.dtype != t0.dtype or not t.is_contiguous() for t in ts):
        return None
    off = t0.data_ptr()
    sp = t0.untyped_storage().data_ptr()
    for t in ts:
        if t.data_ptr() != off or t.untyped_storage().data_ptr() != sp:     # back to back in ONE storage
            return None
        off += t.numel() * t.element_size()
    return t0.as_strided((sum(t.numel() for t in ts),), (1,))


N.register("mdtf_copy2d_multi", [N.P, N.I, N.I, N.P])


class _WeightCats(object):
    """The concatenated ``[K, sum N_i]`` bf16 weights of every multi-weight dense layer (BERT's q|k|v), refreshed by
    ONE batched copy kernel per training step instead of a ``torch.cat`` per layer (12 launches -> 1 for BERT-base).

    Same life cycle as ``ops.conv._FilterTransposes``: the weight shadows change only in the optimizer update, so a
    step marks the copies stale at its start; the first group a step's forward asks for refreshes every group
    registered in earlier steps.  A group seen for the first time is concatenated on its own and registered (not
    inside a graph capture).  Outside a step nothing is cached."""

    def __init__(self):
        self.entries = {}          # tuple of (data_ptr, shape) -> (weights, cat buffer)
        self.order = []
        self.desc = None
        self.blocks = 0
        self.active = False
        self.fresh = False

    def clear(self):
        self.entries.clear()
        del self.order[:]
        self.desc = None
        self.blocks = 0
        self.fresh = False

    def step_begin(self):
        self.active = os.environ.get("MDTF_WEIGHT_CAT_CACHE", "1") != "0"
        self.fresh = False

    def step_end(self):
        self.active = False
        self.fresh = False

    def _rebuild(self):
        import struct
        recs, block = [], 0
        for key in self.order:
            ws, cat = self.entries[key]
            ld = cat.shape[1] // 8
            col = 0
            for w in ws:
                rows, vc = w.shape[0], w.shape[1] // 8
                recs.append(struct.pack("<qqiiiiii", w.data_ptr(), cat.data_ptr() + col * 2, rows, vc, vc, ld,
                                        block, 0))
                block += -(-rows * vc // 1024)
                col += w.shape[1]
        raw = torch.frombuffer(bytearray(b"".join(recs)), dtype=torch.uint8)
        self.desc = raw.to(self.entries[self.order[0]][1].device)
        self.blocks = block
        self.nrec = len(recs)

    def get(self, ws):
        if not self.active or len(ws) < 2:
            return None
        w0 = ws[0]
        if not (w0.is_cuda and all(w.dtype == torch.bfloat16 and w.is_contiguous() and w.dim() == 2
                                   and w.shape[0] == w0.shape[0] and w.shape[1] % 8 == 0 for w in ws)):
            return None
        key = tuple((w.data_ptr(), tuple(w.shape)) for w in ws)
        ent = self.entries.get(key)
        if ent is None:
            from . import conv as _conv
            if torch.cuda.is_current_stream_capturing() or not all(_conv._WT._is_shadow(w) for w in ws):
                return None                      # no new registrations inside a graph capture
            cat = torch.cat(ws, 1)
            self.entries[key] = (tuple(ws), cat)
            self.order.append(key)
            self.desc = None
            return cat
        if not self.fresh:
            if self.desc is None:
                if torch.cuda.is_current_stream_capturing():
                    return None
                self._rebuild()
            N.check(N.fn("mdtf_copy2d_multi")(N.ptr(self.desc), self.nrec, self.blocks, N.stream_ptr()),
                    "copy2d_multi")
            self.fresh = True
        return ent[1]


_CATS = _WeightCats()


class _Dense(torch.autograd.Function):
    """y = act(x @ [W_1 | ... | W_n] + [b_1 | ... | b_n]); ``trans``: W given as [N, K].

    ``x_sink``: the activation-gradient sink of a fanned-out input (a LayerNorm output that also
    feeds the next residual): dx is accumulated into it by the GEMM itself (beta = 1) instead of
    autograd adding two gradient tensors."""

    @staticmethod
    def forward(ctx, x, act, trans, nw, x_sink, x_shape, link_out, link_in, *wb):
        tunable.ensure(x.device)
        ws, bs = wb[:nw], wb[nw:]
        has_b = bs[0] is not None
        ctx.x_sink, ctx.x_shape = x_sink, x_shape
        if x_sink is not None:
            x_sink.register()
        ctx.pp = False
        core = PP_FWD == "all" or (PP_FWD == "fused" and (act != 0 or nw > 1)) or (PP_FWD == "act" and act != 0)
        if not core and PP_FWD_SHAPES and not trans:
            core = "%dx%d" % (x.shape[1], sum(w.shape[1] for w in ws)) in PP_FWD_SHAPES
        if PP and (core or PP_FWD != "act") and x.is_cuda and x.dtype == torch.bfloat16 and x.stride(1) == 1 \
                and N.use_native(x):
            y = None
            if not trans and all(w.is_contiguous() and w.dtype == torch.bfloat16 for w in ws):
                if core:
                    pre = torch.empty((x.shape[0], ws[0].shape[1] * nw), dtype=x.dtype, device=x.device) \
                        if act == 2 else None
                    bl = [t if t.dtype == x.dtype else t.to(x.dtype) for t in bs] if has_b else None
                    y = mm.fwd(x, list(ws), biases=bl, act=act, pre=pre)
                    if y is not None:
                        saved = pre if act == 2 else (y if act == 1 else None)
                if y is None:                            # hipBLASLt (bias epilogue) + the activation kernel
                    w = ws[0] if nw == 1 else _CATS.get(ws)
                    if w is None:
                        w = torch.cat(ws, 1)
                    if has_b:
                        b = bs[0] if nw == 1 else _adjacent(bs)
                        b = (b if b is not None else torch.cat(bs, 0)).to(x.dtype)
                        pre = torch.addmm(b, x, w)
                    else:
                        pre = torch.mm(x, w)
                    y = pre if act == 0 else _act_fwd(pre, act)
                    saved = None if act == 0 else (pre if act == 2 else y)
            elif trans and nw == 1 and act == 0 and ws[0].is_contiguous() and ws[0].dtype == torch.bfloat16:
                y = mm.dgrad(x, ws[0]) if PP_FWD == "all" else None     # x @ w^T, w [N, K]: the dgrad layout
                if y is not None and has_b:
                    y.add_(bs[0].to(y.dtype))
                saved = None
            if y is not None:
                ctx.pp = True
                ctx.act, ctx.trans, ctx.nw, ctx.has_b = act, trans, nw, has_b
                ctx.link_out, ctx.link_in = link_out, link_in
                if link_out is not None:
                    link_out.pre, link_out.act, link_out.fused = saved, act, False
                ctx.widths = [t.shape[0] if trans else t.shape[1] for t in ws]
                ctx.wsinks = [V.grad_sink(t) for t in ws]
                ctx.bsinks = [V.grad_sink(t) if t is not None else None for t in bs]
                ctx.like = wb
                ctx.save_for_backward(x, saved)
                return y
        if has_b:
            b = bs[0] if nw == 1 else _adjacent(bs)
            b = (b if b is not None else torch.cat(bs, 0)).to(x.dtype)
        else:
            b = None
        hand = None if trans else hand_fwd(x, ws, b, act)
        if hand is not None:
            y, pre = hand
            saved = pre if act == 2 else (y if act == 1 else None)
            w = ws[0] if nw == 1 else None          # the data gradient reads the segments in place
        else:
            w = ws[0] if nw == 1 else _CATS.get(ws)
            if w is None:
                w = torch.cat(ws, 1)
            if trans:
                w = w.t()
            pre = torch.addmm(b, x, w) if has_b else torch.mm(x, w)
            if act == 0:
                y, saved = pre, None
            else:
                y = _act_fwd(pre, act)
                saved = pre if act == 2 else y
        ctx.act, ctx.trans, ctx.nw, ctx.has_b = act, trans, nw, has_b
        ctx.link_out, ctx.link_in = link_out, link_in
        if link_out is not None:
            link_out.pre, link_out.act, link_out.fused = saved, act, False
        ctx.widths = [t.shape[0] if trans else t.shape[1] for t in ws]
        ctx.wsinks = [V.grad_sink(t) for t in ws]
        ctx.bsinks = [V.grad_sink(t) if t is not None else None for t in bs]
        ctx.like = wb
        ctx.save_for_backward(x, w, saved)
        return y

    @staticmethod
    def backward(ctx, dy):
        if ctx.pp:
            return _Dense._backward_pp(ctx, dy)
        x, w, saved = ctx.saved_tensors
        if w is None:                             # hand-written forward over q|k|v segments
            w = torch.cat(ctx.like[:ctx.nw], 1)
        dy = dy.contiguous()
        lo = ctx.link_out
        fused_in = lo is not None and lo.fused          # the consumer's dgrad applied act' already
        dpre = dy if (ctx.act == 0 or fused_in) else _act_bwd(dy, saved, ctx.act)
        if lo is not None:
            lo.pre = None
        dx = None
        if ctx.needs_input_grad[0]:
            xs = ctx.x_sink
            hand = not ctx.trans
            li = ctx.link_in
            if xs is None and li is not None and li.pre is not None and hand and ctx.nw == 1:
                if ACT_DGRAD_CORE:                     # the GEMM core's dgrad with the act-backward epilogue
                    dx = mm.dgrad(dpre, w, act_pre=li.pre, act_bwd=li.act)
                else:
                    dx = hand_dgrad_act(dpre, w, li.pre, li.act)      # ffn(): dx already carries act'(pre)
                li.fused = dx is not None
            if dx is None and xs is None:
                dx = _hand_dgrad(dpre, w) if hand else None
                if dx is None:
                    dx = torch.mm(dpre, w.t())
            elif dx is None:
                buf, acc = xs.target()
                if acc:                        # second contribution: C += dpre @ w^T inside the GEMM
                    b2 = buf.view(-1, w.shape[0])
                    if not hand or _hand_dgrad(dpre, w, out=b2, accumulate=True) is None:
                        torch.addmm(b2, dpre, w.t(), out=b2)
                    xs.written(buf)
                else:
                    d2 = _hand_dgrad(dpre, w) if hand else None
                    xs.written((d2 if d2 is not None else torch.mm(dpre, w.t())).view(ctx.x_shape))
        ws, bs = ctx.like[:ctx.nw], ctx.like[ctx.nw:]
        with _wgrad_section(ctx, x, dpre):
            gws, gbs = _Dense._weight_grads(ctx, x, dpre, ws, bs)
        return (dx, None, None, None, None, None, None, None) + tuple(gws) + tuple(gbs)

    @staticmethod
    def _weight_grads(ctx, x, dpre, ws, bs):
        if _wg_backward(ctx, x, dpre):
            return ([V.grad_marker(w) for w in ws],
                    [V.grad_marker(b) for b in bs] if ctx.has_b else [None] * ctx.nw)
        gws, gbs = [], []
        bias_done = [False] * ctx.nw
        col = 0
        for j, n in enumerate(ctx.widths):
            d = dpre[:, col:col + n] if ctx.nw > 1 else dpre
            col += n
            sink = ctx.wsinks[j]
            if sink is not None:
                if ctx.trans:
                    _accum_mm(sink.grad, d.t(), x)
                else:
                    bsink = ctx.bsinks[j] if ctx.has_b else None
                    if wgrad_into(sink.grad, x, d, bsink.grad if bsink is not None else None):
                        bias_done[j] = True
                gws.append(V.grad_marker(ws[j]))
            elif ctx.needs_input_grad[8 + j]:
                g = torch.mm(d.t(), x) if ctx.trans else torch.mm(x.t(), d)
                gws.append(g.to(ws[j].dtype))
            else:
                gws.append(None)
        if ctx.has_b and all(bias_done):
            gbs = [V.grad_marker(b) for b in bs]    # summed inside the weight-gradient kernel
        elif ctx.has_b and any(bias_done):
            tot = kernels.colsum(dpre)
            col = 0
            for j, n in enumerate(ctx.widths):
                part = tot[col:col + n]
                col += n
                if bias_done[j]:
                    gbs.append(V.grad_marker(bs[j]))
                elif ctx.bsinks[j] is not None:
                    ctx.bsinks[j].grad.add_(part)
                    gbs.append(V.grad_marker(bs[j]))
                else:
                    gbs.append(part.to(bs[j].dtype))
        elif ctx.has_b:
            fused = None
            if ctx.nw > 1 and all(sk is not None for sk in ctx.bsinks):
                fused = _adjacent([sk.grad for sk in ctx.bsinks])     # q|k|v slots back to back
            if ctx.nw == 1 and ctx.bsinks[0] is not None:
                kernels.colsum_into(dpre, ctx.bsinks[0].grad)
                gbs.append(V.grad_marker(bs[0]))
            elif fused is not None:
                kernels.colsum_into(dpre, fused)
                gbs = [V.grad_marker(b) for b in bs]
            else:
                tot = kernels.colsum(dpre)
                col = 0
                for j, n in enumerate(ctx.widths):
                    part = tot[col:col + n]
                    col += n
                    if ctx.bsinks[j] is not None:
                        ctx.bsinks[j].grad.add_(part)
                        gbs.append(V.grad_marker(bs[j]))
                    else:
                        gbs.append(part.to(bs[j].dtype))
        else:
            gbs = [None] * ctx.nw
        return gws, gbs


def _pp_weight_grads(ctx, x, dpre, ws, bs):
    """Weight (+ bias) gradients of the core backward, straight into the fp32 slots."""
    wsinks, bsinks = ctx.wsinks, ctx.bsinks
    gws, gbs = [None] * ctx.nw, [None] * ctx.nw
    all_w = all(sk is not None for sk in wsinks)
    all_b = ctx.has_b and all(sk is not None for sk in bsinks)
    done = False
    if _wg_backward(ctx, x, dpre):
        done = True
    elif all_w and (all_b or not ctx.has_b) and PP_WGRAD == "all":
        if ctx.trans:                                   # w [N, K]: g += dy^T x  (C rows = N)
            done = ctx.nw == 1 and mm.wgrad_into([wsinks[0].grad], dpre, x, dbs=None)
            if done and ctx.has_b:
                kernels.colsum_into(dpre, bsinks[0].grad)
        else:
            done = mm.wgrad_into([sk.grad for sk in wsinks], x, dpre,
                                 dbs=[sk.grad for sk in bsinks] if ctx.has_b else None)
    if done:
        gws = [V.grad_marker(w) for w in ws]
        if ctx.has_b:
            gbs = [V.grad_marker(b) for b in bs]
    else:
        col = 0
        for j, n in enumerate(ctx.widths):
            d = dpre[:, col:col + n] if ctx.nw > 1 else dpre
            col += n
            sink = wsinks[j]
            bias_done = False
            if sink is not None:
                if ctx.trans:
                    _accum_mm(sink.grad, d.t(), x)
                else:                                   # conv-kernel wgrad, bias gradient fused in
                    bsk = bsinks[j] if ctx.has_b else None
                    bias_done = wgrad_into(sink.grad, x, d, bsk.grad if bsk is not None else None)
                gws[j] = V.grad_marker(ws[j])
            elif ctx.needs_input_grad[8 + j]:
                g = torch.mm(d.t(), x) if ctx.trans else torch.mm(x.t(), d)
                gws[j] = g.to(ws[j].dtype)
            if ctx.has_b and bias_done:
                gbs[j] = V.grad_marker(bs[j])
            elif ctx.has_b and bsinks[j] is not None:
                kernels.colsum_into(d, bsinks[j].grad) if d.is_contiguous() else bsinks[j].grad.add_(d.float().sum(0))
                gbs[j] = V.grad_marker(bs[j])
            elif ctx.has_b:
                gbs[j] = d.float().sum(0).to(bs[j].dtype)
    return gws, gbs


def _backward_pp(ctx, dy):
    """Backward of a dense layer on the ping-pong core: no weight concatenation, no bf16 weight gradient,
    no separate bias column sums or activation-backward pass where the neighbouring GEMM can fold it in."""
    x, saved = ctx.saved_tensors
    ws, bs = list(ctx.like[:ctx.nw]), list(ctx.like[ctx.nw:])
    dy = dy.contiguous()
    lo = ctx.link_out
    fused_in = lo is not None and lo.fused          # the consumer's data gradient applied act' already
    dpre = dy if (ctx.act == 0 or fused_in) else _act_bwd(dy, saved, ctx.act)
    if lo is not None:
        lo.pre = None
    dx = None
    if ctx.needs_input_grad[0]:
        xs, li = ctx.x_sink, ctx.link_in
        if ctx.trans:                                   # y = x w^T (w [N, K]): dx = dy w
            w = ws[0]
            dx = mm.fwd(dpre, w) if dpre.shape[1] % 64 == 0 else None
            if dx is None:
                dx = torch.mm(dpre, w)
            if xs is not None:
                buf, acc = xs.target()
                if acc:
                    buf.view(-1, dx.shape[1]).add_(dx)
                    xs.written(buf)
                else:
                    xs.written(dx.view(ctx.x_shape))
                dx = None
        elif xs is None:
            ap = li.pre if (li is not None and li.pre is not None) else None
            core = PP_DGRAD == "all" or (PP_DGRAD == "fused" and (ap is not None or ctx.nw > 1)) or \
                _dgrad_shape_on(ws)
            dx = mm.dgrad(dpre, ws, act_pre=ap, act_bwd=li.act if ap is not None else 0) if core else None
            if dx is not None and ap is not None:
                li.fused = True
            if dx is None:
                w = ws[0] if ctx.nw == 1 else torch.cat(ws, 1)
                dx = torch.mm(dpre, w.t())
        else:
            buf, acc = xs.target()
            K = ws[0].shape[0]
            core = PP_DGRAD == "all" or (PP_DGRAD == "fused" and ctx.nw > 1) or _dgrad_shape_on(ws)
            if acc:                                     # second contribution: C += dpre @ w^T inside the GEMM
                b2 = buf.view(-1, K)
                if not core or mm.dgrad(dpre, ws, out=b2, accumulate=True) is None:
                    torch.addmm(b2, dpre, torch.cat(ws, 1).t() if ctx.nw > 1 else ws[0].t(), out=b2)
                xs.written(buf)
            else:
                d2 = mm.dgrad(dpre, ws) if core else None
                if d2 is None:
                    d2 = torch.mm(dpre, torch.cat(ws, 1).t() if ctx.nw > 1 else ws[0].t())
                xs.written(d2.view(ctx.x_shape))
    # weight (+ bias) gradients straight into the fp32 slots
    with _wgrad_section(ctx, x, dpre):
        gws, gbs = _pp_weight_grads(ctx, x, dpre, ws, bs)
    return (dx, None, None, None, None, None, None, None) + tuple(gws) + tuple(gbs)


_Dense._backward_pp = staticmethod(_backward_pp)


def matmul(a, b):
    return torch.matmul(a, b)


def _check(x, what):
    if x.dtype != torch.bfloat16:
        raise TypeError("mdtf %s expects bf16 activations on the GPU, got %s" % (what, x.dtype))


def dense(x, w, b=None, act=None):
    """``act(x @ w + b)`` for x [..., K], w [K, N]."""
    return dense_multi(x, [w], [b], act)


def dense_multi(x, ws, bs, act=None):
    """One GEMM for several weight matrices sharing input ``x`` (outputs concatenated)."""
    _check(x, "dense")
    from . import actsink
    shp = x.shape
    x2 = x.reshape(-1, shp[-1])
    ws = [w.to(x.dtype) if w.dtype != x.dtype else w for w in ws]
    y = _Dense.apply(x2, _ACT[act], False, len(ws), actsink.sink_of(x), tuple(shp), None, None, *ws, *bs)
    return y.reshape(*shp[:-1], y.shape[-1])


# MDTF_DEC_SPLIT: split-K chunks of the padded tied decoder's data gradient (0: the plain dense_transposed path)
DEC_SPLIT = int(os.environ.get("MDTF_DEC_SPLIT", "8"))
_PADDED_GRADS = {}     # data_ptr -> row stride of zero-padded logit gradients made by kernels._Xent


def decoder_pad_rows(vocab, split=None):
    """Zero rows to reserve after a tied [vocab, H] embedding so the decoder's vocabulary splits into ``split``
    chunks of whole 256-row blocks (BERT: 30522 -> 30720 = 8 x 3840)."""
    split = DEC_SPLIT if split is None else split
    q = 256 * max(split, 1)
    return (-vocab) % q


class _TiedDecoder(torch.autograd.Function):
    """``logits = h W^T + b`` of a tied MLM decoder over the vocabulary padded to the variables' ``pad_rows``
    (parallel/flat.py keeps the pad rows of master, gradient and bf16 shadow at zero), reference
    ``distribute_tools.py:204-206`` (tf.matmul + bias_add of FC_layer; BERT's decoder is that product against the
    transposed embedding).  Padded, the three products leave the library's odd-width tiles:

      forward   logits_p = b_p + h W_p^T       [rows, VP]; the model sees the [rows, V] view
      dgrad     dh = sum_s dlogits_p[:, s] W_p[s]   split-K over DEC_SPLIT vocabulary chunks as one batched
                product with fp32 partials (80 output tiles unsplit: profiles/mlm_decoder_r5.md)
      wgrad     gW_p += dlogits_p^T h  and  gb_p += colsum(dlogits_p), straight into the padded fp32 slots

    The logit gradient arrives as the [rows, V] view of the zero-padded [rows, VP] buffer kernels._Xent writes for
    strided logits; any other producer's gradient is copied into a zero-padded buffer first."""

    @staticmethod
    def forward(ctx, h, w, b):
        wv, bv = w._mdtf_var, b._mdtf_var
        Wp = wv.shadow_padded
        bp = bv.shadow_padded if bv.shadow_padded is not None else bv.master_padded.to(h.dtype)
        Vn = wv.shape[0]
        logits = torch.addmm(bp, h, Wp.t())
        ctx.save_for_backward(h)
        ctx.wv, ctx.bv, ctx.V = wv, bv, Vn
        ctx.like = (w, b)
        return logits[:, :Vn]

    @staticmethod
    def backward(ctx, dy):
        h, = ctx.saved_tensors
        wv, bv, Vn = ctx.wv, ctx.bv, ctx.V
        Wp = wv.shadow_padded
        VP, H = Wp.shape
        M = h.shape[0]
        base = dy._base
        if (dy.stride(1) == 1 and dy.stride(0) == VP and base is not None and tuple(base.shape) == (M, VP)
                and base.data_ptr() == dy.data_ptr() and _PADDED_GRADS.pop(dy.data_ptr(), None) == VP):
            dp = base                      # the zero-padded [rows, VP] buffer kernels._Xent wrote
        else:
            dp = torch.zeros((M, VP), dtype=h.dtype, device=h.device)
            dp[:, :Vn].copy_(dy)
        S = DEC_SPLIT
        try:
            part = torch.bmm(dp.view(M, S, VP // S).transpose(0, 1), Wp.view(S, VP // S, H), out_dtype=torch.float32)
            dh = part.sum(0).to(h.dtype)
        except (RuntimeError, TypeError):
            dh = torch.mm(dp, Wp)
        # the decoder's weight gradient writes the whole (padded) slot: as the step's first writer it overwrites it
        # (V.claim_store; the word embedding's scatter-add accumulates onto it later)
        _accum_mm(wv.grad_padded, dp.t(), h, store=V.claim_store(wv))
        kernels.colsum_into(dp, bv.grad_padded)
        w, b = ctx.like
        return dh, V.grad_marker(w), V.grad_marker(b)


def tied_decoder(x, w, b):
    """``x @ w^T + b`` for a tied decoder: the padded path when both variables carry padded flat views (set
    ``pad_rows`` from :func:`decoder_pad_rows` before the flat space is built), else :func:`dense_transposed`."""
    wv, bv = getattr(w, "_mdtf_var", None), getattr(b, "_mdtf_var", None)
    ok = (DEC_SPLIT > 0 and wv is not None and bv is not None and x.dim() == 2 and x.is_cuda
          and x.dtype == torch.bfloat16 and wv.shadow_padded is not None and wv.grad_padded is not None
          and bv.grad_padded is not None and (bv.shadow_padded is not None or bv.master_padded is not None)
          and wv.shadow_padded.shape[0] == bv.grad_padded.shape[0]
          and wv.shadow_padded.shape[0] % (256 * DEC_SPLIT) == 0 and torch.is_grad_enabled()
          and V.grad_sink(w) is wv and V.grad_sink(b) is bv)
    if not ok:
        return dense_transposed(x, w, b)
    _check(x, "dense")
    return _TiedDecoder.apply(x.contiguous(), w, b)


def dense_transposed(x, w, b=None):
    """``x @ w^T + b`` with w [N, K] (tied embedding decoders)."""
    _check(x, "dense")
    shp = x.shape
    w = w.to(x.dtype) if w.dtype != x.dtype else w
    y = _Dense.apply(x.reshape(-1, shp[-1]), 0, True, 1, None, tuple(shp), None, None, w, b)
    return y.reshape(*shp[:-1], y.shape[-1])


def ffn(x, w1, b1, w2, b2, act="gelu"):
    """``act(x @ w1 + b1) @ w2 + b2`` (a transformer feed-forward block).  The intermediate has exactly one
    consumer, so the second layer's data gradient applies the activation derivative in its epilogue
    (:func:`hand_dgrad_act`) and the first layer skips its activation-backward pass."""
    _check(x, "ffn")
    from . import actsink
    shp = x.shape
    x2 = x.reshape(-1, shp[-1])
    w1 = w1.to(x.dtype) if w1.dtype != x.dtype else w1
    w2 = w2.to(x.dtype) if w2.dtype != x.dtype else w2
    link = _ActLink() if (FFN_FUSE and _ACT[act] != 0) else None
    h = _Dense.apply(x2, _ACT[act], False, 1, actsink.sink_of(x), tuple(shp), link, None, w1, b1)
    y = _Dense.apply(h, 0, False, 1, None, tuple(h.shape), None, link, w2, b2)
    return y.reshape(*shp[:-1], y.shape[-1])
