"""Convolution on the GPU: hand-written implicit-GEMM MFMA kernels (``csrc/conv_igemm.hip``).

NHWC activations, HWIO filters (TF layouts, which are also the natural
implicit-GEMM layouts: ``W[(kh,kw,ci)][co]`` is the row-major B matrix).
Each pass (fwd / dgrad / wgrad) of each conv shape runs on the backend chosen
by the per-shape table ``conv_table.json`` (written by
``bench/conv_autotune.py`` on an MI355X: the hand-written kernel wherever it
beats MIOpen, with its best tile); ``MDTF_CONV=mdtf|miopen`` forces one
backend.  Shapes the HIP kernel cannot take (C % 8 != 0, e.g. a 3-channel
stem) use MIOpen.
"""
import ctypes
import json
import os

import torch
import torch.nn.functional as F

from . import _native as N
from . import winograd
from ..train import variables as V

N.register("mdtf_conv_fwd", [N.P, N.P, N.P, N.P, N.P] + [N.I] * 18 + [N.P, N.P])
N.register("mdtf_conv_dgrad", [N.P, N.P, N.P] + [N.I] * 17 + [N.P])
N.register("mdtf_conv_wgrad", [N.P, N.P, N.P] + [N.I] * 18 + [N.P])
N.register("mdtf_conv_fwd_v2", [N.P, N.P, N.P, N.P, N.P] + [N.I] * 18 + [N.P, N.P])
N.register("mdtf_conv_dgrad_v2", [N.P, N.P, N.P] + [N.I] * 18 + [N.P, N.P, N.P, N.P, N.I, N.P, N.P, N.P])
N.register("mdtf_conv_wgrad_v2", [N.P, N.P, N.P] + [N.I] * 18 + [N.P, N.I, N.P])
N.register("mdtf_set_slab_stream", [N.P])
N.register("mdtf_set_wgrad_store", [N.I])
N.register("mdtf_set_wgrad_fin", [N.P, N.P, N.I, N.P, N.P, N.P, N.P, N.L, N.I])

# split-K weight gradients: per-split partial slabs + one reduction pass (plain stores) instead of fp32
# atomics into DW.  Measured on MI355X (scripts/gpu.sh envab): +0.4 % BERT-base (dense GEMM weight
# gradients), -0.3 % ResNet-50 (conv tiles were autotuned with atomics) -> default: dense layers only.
# MDTF_WGRAD_SLAB = dense (default) | 1 (conv too) | 0 (atomics everywhere)
_SLAB_MODE = os.environ.get("MDTF_WGRAD_SLAB", "dense")
WGRAD_SLAB = _SLAB_MODE not in ("0", "", "false", "dense")
DENSE_WGRAD_SLAB = _SLAB_MODE not in ("0", "", "false")


def wgrad_splits(M, R, Cout, bm, bn, ver, splits):
    """The split count launch_wgrad_v2 (csrc/conv_igemm.hip) will use."""
    kt_total = -(-M // 64)
    tiles = -(-R // bm) * -(-Cout // bn)
    if splits < 1:
        splits = -(-(512 if ver == 3 else 1024) // tiles)
    splits = max(1, min(splits, kt_total))
    ks = -(-kt_total // splits)
    return -(-kt_total // ks)


def wgrad_slab(M, R, Cout, bm, bn, ver, splits, device, dense=False, force=None):
    """(slab tensor or None, capacity) for one v2 weight-gradient launch.  ``force``: a per-shape choice of the
    conv table (``"slab"`` field) over the global MDTF_WGRAD_SLAB default."""
    on = (DENSE_WGRAD_SLAB if dense else WGRAD_SLAB) if force is None else force
    if not on or N.deterministic():
        return None, 0
    sp = wgrad_splits(M, R, Cout, bm, bn, ver, splits)
    if sp < 2:
        return None, 0
    if WGRAD_INK:     # in-kernel reduction: [tiles][splits][BM * BN] partial tiles, tiles padded to 256 multiples
        return torch.empty(sp * (-(-R // 256) * 256) * (-(-Cout // 256) * 256), dtype=torch.float32,
                           device=device), sp
    return torch.empty(sp * R * Cout, dtype=torch.float32, device=device), sp


# MDTF_WGRAD_INK=1: split-K weight gradients summed inside the kernel by each tile's last arriving workgroup
# (write-through partial tiles + one ticket per workgroup, csrc/conv_igemm.hip) instead of slab stores + a
# wgrad_slab_reduce launch.  Correct, but -12.5 % ResNet-50 / -1.3 % BERT in the step (profiles/ab_r6.md): one
# workgroup per tile reads the other splits' partial tiles at ~100 GB/s (a serial tail of several us per tile, 8-128
# splits), where the reduction launch spreads the same bytes over every CU.  Off.
WGRAD_INK = os.environ.get("MDTF_WGRAD_INK", "0") == "1"
N.register("mdtf_set_wgrad_tickets", [N.P, N.L])


class wgrad_tickets:
    """Context for one native v2 weight-gradient launch with a slab: hands it this stream's zeroed per-tile tickets
    (``ops.mm._tickets``: one buffer per (device, stream), every launch leaves its tickets at zero)."""

    def __init__(self, slab):
        self.on = WGRAD_INK and slab is not None and slab.is_cuda
        self.device = slab.device if self.on else None

    def __enter__(self):
        if self.on:
            from . import mm
            t = mm._tickets(self.device, 4096)
            N.fn("mdtf_set_wgrad_tickets")(N.ptr(t), t.numel())
        return self

    def __exit__(self, *exc):
        if self.on:
            N.fn("mdtf_set_wgrad_tickets")(None, 0)
        return False

_HERE = os.path.dirname(os.path.abspath(__file__))
TUNED_BATCH = 256        # the batch bench/conv_autotune.py tuned conv_table.json at
TABLE_PATH = os.environ.get("MDTF_CONV_TABLE") or os.path.join(_HERE, "conv_table.json")
_TABLE = None


def table():
    global _TABLE
    if _TABLE is None:
        _TABLE = {}
        if os.path.exists(TABLE_PATH):
            with open(TABLE_PATH) as f:
                _TABLE = json.load(f)
    return _TABLE


def shape_key(pass_, x_shape, w_shape, stride, pads, dil):
    n, h, w, c = x_shape
    kh, kw, ci, co = w_shape
    return "%s:%d,%d,%d,%d:%d,%d,%d:%d,%d:%d,%d,%d,%d:%d,%d" % (
        pass_, n, h, w, c, kh, kw, co, stride[0], stride[1], pads[0], pads[1], pads[2], pads[3], dil[0], dil[1])


def _default_tile(ncol):
    return (128, 128) if ncol % 128 == 0 else (128, 64)


def v2_ok(pass_, c, co, stride=(1, 1), taps=1, dil=(1, 1)):
    """The BK=64 LDS-DMA kernels: gathered channels % 64 == 0, <= 32 filter taps; strided dgrad undilated."""
    if taps > 32:
        return False
    if pass_ == "fwd":
        return c % 64 == 0 and co % 8 == 0
    if pass_ == "dgrad":
        return co % 64 == 0 and c % 8 == 0 and (tuple(stride) == (1, 1) or tuple(dil) == (1, 1))
    if pass_ == "wgrad":
        return c % 64 == 0 and co % 64 == 0
    return False


def choose(pass_, x_shape, w_shape, stride, pads, dil):
    """-> ('mdtf', bm, bn, splits, version, stages), ('ws', (tp, nw, cg, d)) (the weight-stationary
    kernel, csrc/conv_ws.hip), ('winograd',) or ('miopen',).

    ``MDTF_CONV``: ``auto`` (table, else defaults), ``mdtf`` (v1 kernels),
    ``mdtf2`` (v2 kernels where the channels allow, else v1), ``miopen``.
    """
    n, h, w, c = x_shape
    kh, kw, ci, co = w_shape
    forced = os.environ.get("MDTF_CONV", "auto")
    native_ok = c % 8 == 0 and co % 8 == 0
    if pass_ in ("fwd", "wgrad") and not native_ok and stem_ok(x_shape, w_shape, dil):
        if pass_ == "fwd" or (co == 64 and kh <= 8 and not N.deterministic()):
            return ("stem",)
    if not native_ok or forced == "miopen":
        return ("miopen",)
    if pass_ in ("fwd", "dgrad") and winograd.enabled() and winograd.eligible(w_shape, stride, pads, dil, c, co):
        return ("winograd",)                 # the reference's TF_ENABLE_WINOGRAD_NONFUSED toggle
    ent = table().get(shape_key(pass_, x_shape, w_shape, stride, pads, dil))
    if ent is None and n != TUNED_BATCH:
        # batch-agnostic lookup: the same conv at the tuned batch (ResNet-50/101/152 share their conv
        # shapes; e.g. the async-PS ResNet-152 at batch 64 takes the batch-256 choices)
        ent = table().get(shape_key(pass_, (TUNED_BATCH, h, w, c), w_shape, stride, pads, dil))
    if N.deterministic() and pass_ == "wgrad":
        # no split-K atomics, no library algorithm choice: one block per DW tile
        ver = 2 if v2_ok(pass_, c, co, stride, kh * kw, dil) else 1
        return ("mdtf", 128 if kh * kw * ci >= 128 else 64, 128 if co % 128 == 0 else 64, 1, ver, 2)
    if forced == "auto" and ent is not None:
        if ent["backend"] in ("miopen", "winograd"):
            return (ent["backend"],)
        if ent.get("ver") == 5:                  # ping-pong core (csrc/gemm_pp.hip mdtf_conv_pp)
            if pp_ok(pass_, c, co, stride, kh, kw, ent["tile"]):
                return ("pp", ent["tile"])
            ent = ent.get("prev")
            if ent is None:
                return ("mdtf",) + _default_tile(co if pass_ == "fwd" else ci) + (0, 2, 2)
            if ent["backend"] in ("miopen", "winograd"):
                return (ent["backend"],)
        if ent.get("ver") == 4:
            if N.deterministic():                # cross-block statistics atomics: use the v2 kernels
                return ("mdtf", 128, 128 if (co if pass_ == "fwd" else c) % 128 == 0 else 64, 0, 2, 2)
            return ("ws", tuple(ent["ws"]))
        return ("mdtf", ent["bm"], ent["bn"], ent.get("splits", 0), ent.get("ver", 1), ent.get("stages", 2))
    if pass_ == "wgrad":
        r = kh * kw * ci
        ver = 2 if (forced in ("auto", "mdtf2") and v2_ok(pass_, c, co, stride, kh * kw, dil)) else 1
        return ("mdtf", 128 if r >= 128 else 64, 128 if co % 128 == 0 else 64, 0, ver, 2)
    ncol = co if pass_ == "fwd" else ci
    bm, bn = _default_tile(ncol)
    ver = 2 if (forced in ("auto", "mdtf2") and v2_ok(pass_, c, co, stride, kh * kw, dil)) else 1
    return ("mdtf", bm, bn, 0, ver, 3 if ver == 2 else 2)


# ---------------------------------------------------------------------------
# MIOpen (library) path through aten on channels-last views
# ---------------------------------------------------------------------------
def _nchw(x):
    return x.permute(0, 3, 1, 2)


def _w_oihw(w):
    return w.permute(3, 2, 0, 1).contiguous(memory_format=torch.channels_last)


def _sym(pads):
    pt, pb, pl, pr = pads
    return pt == pb and pl == pr


def miopen_fwd(x, w, stride, pads, dil):
    pt, pb, pl, pr = pads
    xc = _nchw(x)
    if not _sym(pads):
        xc = F.pad(xc, (pl, pr, pt, pb))
        pt = pl = 0
    y = F.conv2d(xc, _w_oihw(w).to(x.dtype), None, stride, (pt, pl), dil)
    return y.permute(0, 2, 3, 1).contiguous()


def miopen_bwd(x, w, dy, stride, pads, dil, need_dx, need_dw):
    pt, pb, pl, pr = pads
    xc = _nchw(x)
    if not _sym(pads):
        xc = F.pad(xc, (pl, pr, pt, pb))
        ph, pw = 0, 0
    else:
        ph, pw = pt, pl
    wt = _w_oihw(w).to(x.dtype)
    dyc = _nchw(dy)
    dx_c, dw_c, _ = torch.ops.aten.convolution_backward(
        dyc, xc, wt, None, list(stride), [ph, pw], list(dil), False, [0, 0], 1, [need_dx, need_dw, False])
    dx = dw = None
    if need_dx:
        if not _sym(pads):
            dx_c = dx_c[:, :, pt:pt + x.shape[1], pl:pl + x.shape[2]]
        dx = dx_c.permute(0, 2, 3, 1).contiguous()
    if need_dw:
        dw = dw_c.permute(2, 3, 1, 0).contiguous()       # OIHW -> HWIO
    return dx, dw


# ---------------------------------------------------------------------------
# hand-written kernels
# ---------------------------------------------------------------------------
def _geo(x, w, out_hw, stride, pads, dil):
    n, h, wd, c = x.shape
    kh, kw, ci, co = w.shape
    return [n, h, wd, c, out_hw[0], out_hw[1], co, kh, kw, stride[0], stride[1], pads[0], pads[2], dil[0], dil[1]]


def transpose_filter(w):
    """HWIO [kh,kw,ci,co] -> Wt [co][(kh,kw,ci)] (the v2 forward kernel's K-contiguous B operand)."""
    cached = _WT.get(w)
    if cached is not None:
        return cached
    from . import kernels
    kh, kw, ci, co = w.shape
    return kernels.transpose_brs(w.reshape(1, kh * kw * ci, co), 1, kh * kw * ci, co).view(co, kh * kw * ci)


N.register("mdtf_transpose_multi", [N.P, N.I, N.I, N.P])


class _FilterTransposes(object):
    """All conv filters' K-contiguous copies, refreshed by ONE batched kernel per training step.

    The bf16 filter shadows change only in the optimizer update, so a training step marks the cache stale
    at its start (``step_begin``) and invalid again after the update (``step_end``).  The first filter a
    step's forward asks for launches the batched transpose of every filter registered in earlier steps
    (52 launches -> 1 for ResNet-50); a filter seen for the first time is transposed on its own and
    registered.  Outside a step (eval, checkpoint restore) nothing is cached.
    """

    def __init__(self):
        self.entries = {}          # (data_ptr, shape) -> (filter view, Wt buffer)
        self.order = []
        self.desc = None
        self.tiles = 0
        self.active = False        # inside a training step
        self.fresh = False         # every registered copy is current for this step

    def clear(self):
        """Forget every registered filter (a new model / flat space, a released step graph): dead filters
        must neither stay referenced nor keep being transposed by the batched kernel."""
        self.entries.clear()
        del self.order[:]
        self.desc = None
        self.tiles = 0
        self.fresh = False

    def step_begin(self):
        self.active = os.environ.get("MDTF_FILTER_CACHE", "1") != "0"
        self.fresh = False

    def step_end(self):
        self.active = False
        self.fresh = False

    def _rebuild(self):
        import struct
        recs, tile = [], 0
        for key in self.order:
            w, wt = self.entries[key]
            r = w.numel() // w.shape[-1]
            sdim = w.shape[-1]
            ts = -(-sdim // 64)
            recs.append(struct.pack("<qqqii", w.data_ptr(), wt.data_ptr(), r | (sdim << 32), tile, ts))
            tile += ts * -(-r // 64)
        raw = torch.frombuffer(bytearray(b"".join(recs)), dtype=torch.uint8)
        self.desc = raw.to(self.order and self.entries[self.order[0]][0].device)
        self.tiles = tile

    @staticmethod
    def _is_shadow(w):
        """Only filters living in a flat parameter space's bf16 shadow (stable storage, rewritten in place by
        the optimizer) are cached; per-step temporaries are not."""
        flat = getattr(V.get_store(), "flat", None)
        if flat is None:
            return False
        sp = w.untyped_storage().data_ptr()
        return any(g.shadow is not None and g.shadow.untyped_storage().data_ptr() == sp for g in flat.groups)

    def get(self, w):
        if not self.active or not w.is_cuda or w.dtype != torch.bfloat16 or not w.is_contiguous():
            return None
        key = (w.data_ptr(), tuple(w.shape))
        ent = self.entries.get(key)
        if ent is None:
            if torch.cuda.is_current_stream_capturing() or not self._is_shadow(w):
                return None                      # no new registrations inside a graph capture
            from . import kernels
            kh, kw, ci, co = w.shape
            wt = torch.empty((co, kh * kw * ci), dtype=w.dtype, device=w.device)
            self.entries[key] = (w, wt)
            self.order.append(key)
            self.desc = None
            wt.copy_(kernels.transpose_brs(w.reshape(1, kh * kw * ci, co), 1, kh * kw * ci, co).view(co, -1))
            return wt
        if not self.fresh:
            if self.desc is None:
                if torch.cuda.is_current_stream_capturing():
                    return None
                self._rebuild()
            N.check(N.fn("mdtf_transpose_multi")(N.ptr(self.desc), len(self.order), self.tiles, N.stream_ptr()),
                    "transpose_multi")
            self.fresh = True
        return ent[1]


_WT = _FilterTransposes()


def _v2_code(bm, stages, ver):
    """C-ABI tile code of the v2 kernels: [10000 if 8 waves] + 1000 * stages + tile rows.
    ``ver`` 2 = 4-wave tiles, 3 = 8-wave tiles (one 256-row or 256-column block per CU).  Two-digit stage codes
    (split A/B rings: 10 * A stages + B stages) use 100000 * (1 + [8 waves]) + 1000 * stages + rows."""
    if stages >= 10:
        return bm + 1000 * stages + 100000 * (2 if ver == 3 else 1)
    return bm + 1000 * stages + (10000 if ver == 3 else 0)


def mdtf_fwd(x, w, out_hw, stride, pads, dil, bm, bn, stats=None, ver=1, stages=2):
    n = x.shape[0]
    co = w.shape[3]
    y = torch.empty((n, out_hw[0], out_hw[1], co), dtype=x.dtype, device=x.device)
    mt = N.I(0)
    s_sum, s_sq = (stats if stats is not None else (None, None))
    slots = s_sum.shape[0] if s_sum is not None else 0
    import ctypes
    if ver in (2, 3):
        wt = transpose_filter(w)
        N.check(N.fn("mdtf_conv_fwd_v2")(N.ptr(x), N.ptr(wt), N.ptr(y), N.ptr(s_sum), N.ptr(s_sq), slots,
                                         *_geo(x, w, out_hw, stride, pads, dil), _v2_code(bm, stages, ver), bn,
                                         ctypes.byref(mt),
                                         N.stream_ptr()), "conv_fwd_v2")
        return y
    N.check(N.fn("mdtf_conv_fwd")(N.ptr(x), N.ptr(w), N.ptr(y), N.ptr(s_sum), N.ptr(s_sq), slots,
                                  *_geo(x, w, out_hw, stride, pads, dil), bm, bn, ctypes.byref(mt), N.stream_ptr()),
            "conv_fwd")
    return y


def mdtf_dgrad(dy, w, x_shape, stride, pads, dil, bm, bn, ver=1, stages=2, out=None, accumulate=False,
               bn_stats=None, acc_src=None):
    """DX of a conv; v2 can write into ``out`` and accumulate (out += dgrad) in its epilogue.

    ``bn_stats = (x, relu_mask or None, psum, psq, slots)``: DX is the complete gradient of a BatchNorm
    output; the epilogue also accumulates that BN's backward statistics into ``psum``/``psq``.
    ``acc_src = (g, relu_mask)``: accumulate ``g * mask`` instead of ``out``'s contents (a pending
    masked contribution of an activation-gradient sink, ``actsink``)."""
    dx = out if out is not None else torch.empty(x_shape, dtype=dy.dtype, device=dy.device)
    n, h, wd, c = x_shape
    kh, kw, ci, co = w.shape
    geo = [n, h, wd, c, dy.shape[1], dy.shape[2], co, kh, kw, stride[0], stride[1], pads[0], pads[2], dil[0], dil[1]]
    if ver in (2, 3):
        bx, bmask, bsum, bsq, bslots = bn_stats if bn_stats is not None else (None, None, None, None, 0)
        ag, am = acc_src if acc_src is not None else (None, None)
        N.check(N.fn("mdtf_conv_dgrad_v2")(N.ptr(dy), N.ptr(w), N.ptr(dx), *geo, _v2_code(bm, stages, ver), bn,
                                           int(bool(accumulate) or acc_src is not None), N.ptr(bx), N.ptr(bmask),
                                           N.ptr(bsum), N.ptr(bsq), int(bslots), N.ptr(ag), N.ptr(am),
                                           N.stream_ptr()), "conv_dgrad_v2")
        return dx
    if acc_src is not None:
        raise ValueError("a masked accumulate source needs the v2 kernel")
    if bn_stats is not None:
        raise ValueError("BN statistics in the dgrad epilogue need the v2 kernel")
    if accumulate:
        raise ValueError("accumulating dgrad needs the v2 kernel")
    N.check(N.fn("mdtf_conv_dgrad")(N.ptr(dy), N.ptr(w), N.ptr(dx), *geo, bm, bn, N.stream_ptr()), "conv_dgrad")
    return dx


N.register("mdtf_conv_ws", [N.P, N.P, N.P] + [N.I] * 16 + [N.I, N.I] +
           [N.P, N.P, N.I, N.P, N.P, N.P, N.P, N.I, N.I, N.P, N.P, N.P])


def ws_ok(pass_, c, co, stride, kh, kw, dil=(1, 1)):
    """Shapes the weight-stationary kernel (csrc/conv_ws.hip) takes: the reduced channels % 32,
    output channels % 64, the block's filter slice (64 output channels x K) <= 144 KiB of LDS;
    dgrad stride 1 only."""
    if pass_ == "fwd":
        red, ncol = c, co
    elif pass_ == "dgrad":
        if tuple(stride) != (1, 1):
            return False
        red, ncol = co, c
    else:
        return False
    return (red % 32 == 0 and ncol % 64 == 0 and kh * kw <= 32 and kh * kw * red >= 64
            and 64 * kh * kw * red * 2 <= 160 * 1024)


N.register("mdtf_stem_pack4", [N.P, N.P] + [N.I] * 8 + [N.P, N.P] + [N.I] * 4 + [N.P])
N.register("mdtf_conv_ws_stem", [N.P, N.P, N.P] + [N.I] * 10 + [N.P, N.P, N.I, N.P])
N.register("mdtf_stem_conv_rows", [N.P, N.P, N.P] + [N.I] * 10 + [N.P, N.P, N.I, N.P])
N.register("mdtf_stem_wgrad", [N.P, N.P, N.P] + [N.I] * 11 + [N.P])
STEM = os.environ.get("MDTF_STEM", "mdtf")          # mdtf: hand-written stem forward | miopen
# rows: row-staged kernel (both operands from LDS, one output row per wave) | ws: streamed weight-stationary kernel
STEM_KERNEL = os.environ.get("MDTF_STEM_KERNEL", "rows")
_STEM_PACK_W = os.environ.get("MDTF_STEM_PACK_W", "1") != "0"     # filter rows packed in the x4 launch
STEM_TILE = (4, 4, 1, 4)          # bench/stem_ws_probe.py: 0.329 ms vs MIOpen 0.487 (batch 256)


def stem_ok(x_shape, w_shape, dil):
    """Few-channel stems (Cin <= 4, KW <= 8, undilated): csrc/conv_ws.hip mdtf_conv_ws_stem."""
    kh, kw, ci, co = w_shape
    return (STEM != "miopen" and ci <= 4 and kw <= 8 and co % 64 == 0 and tuple(dil) == (1, 1)
            and x_shape[2] * ci <= 16384                          # source row staged in LDS (stem_pack4)
            and os.environ.get("MDTF_CONV", "auto") != "miopen")


# blocks of the stem weight gradient: 3 per CU (78 VGPRs x 8 waves, 40 KB LDS) fill the chip in one round;
# bench/stem_wgrad_probe.py: 256 / 512 / 768 / 1024 blocks -> 362 / 226 / 191 / 222 us
STEM_WG_BLOCKS = int(os.environ.get("MDTF_STEM_WG_BLOCKS", "768"))


def stem_wgrad(x4, dy, w_shape, stride, out=None, blocks=0):
    """Stem weight gradient from the forward's packed x4 (csrc/stem_wgrad.hip): fp32 HWIO, accumulated
    into ``out`` (a zeroed buffer or the variable's gradient slot)."""
    kh, kw, ci, co = w_shape
    dw = out if out is not None else torch.zeros(w_shape, dtype=torch.float32, device=dy.device)
    n, h4, w4, _ = x4.shape
    N.check(N.fn("mdtf_stem_wgrad")(N.ptr(x4), N.ptr(dy), N.ptr(dw), n, h4, w4, dy.shape[1], dy.shape[2],
                                    stride[0], stride[1], kh, kw, ci, int(blocks or STEM_WG_BLOCKS),
                                    N.stream_ptr()), "stem_wgrad")
    return dw


def stem_fwd(x, w, out_hw, stride, pads, stats=None, tile=None, keep_x4=None):
    """Stem forward: repack x into a zero-haloed 4-channel image and the filter into rows [co][row][kw*4 + c]
    (zero-padded; one kernel for both), then the weight-stationary GEMM with one 32-deep k-step per row."""
    n, h, wd, c = x.shape
    kh, kw, ci, co = w.shape
    pt, pb, pl, pr = pads
    khp = -(-kh // 4) * 4
    h4 = max(h + pt + pb, (out_hw[0] - 1) * stride[0] + khp)
    w4 = max(wd + pl + pr, (out_hw[1] - 1) * stride[1] + 8)
    w4 += w4 & 1                                   # even: 16-B aligned rows for the row-staged kernel
    x4 = torch.empty((n, h4, w4, 4), dtype=x.dtype, device=x.device)
    assert ci == c, "stem filter channels %d != input channels %d" % (ci, c)
    w = w.to(x.dtype).contiguous()
    if _STEM_PACK_W:
        wt = torch.empty((co, khp * 32), dtype=x.dtype, device=x.device)      # [co][row][kw*4 + c]
    else:
        wp = torch.zeros((khp, 8, 4, co), dtype=x.dtype, device=x.device)
        wp[:kh, :kw, :ci].copy_(w)
        wt = wp.view(khp * 32, co).t().contiguous()
    N.check(N.fn("mdtf_stem_pack4")(N.ptr(x), N.ptr(x4), n, h, wd, c, pt, pl, h4, w4,
                                    N.ptr(w if _STEM_PACK_W else None), N.ptr(wt), kh, kw, co, khp,
                                    N.stream_ptr()), "stem_pack4")
    y = torch.empty((n, out_hw[0], out_hw[1], co), dtype=x.dtype, device=x.device)
    s_sum, s_sq = stats if stats is not None else (None, None)
    slots = s_sum.shape[0] if s_sum is not None else 0
    if STEM_KERNEL == "rows" and tile is None and out_hw[1] <= 128:
        N.check(N.fn("mdtf_stem_conv_rows")(N.ptr(x4), N.ptr(wt), N.ptr(y), n, h4, w4, out_hw[0], out_hw[1], co, kh,
                                            khp, stride[0], stride[1], N.ptr(s_sum), N.ptr(s_sq), slots,
                                            N.stream_ptr()), "stem_conv_rows")
    else:
        N.check(N.fn("mdtf_conv_ws_stem")(N.ptr(x4), N.ptr(wt), N.ptr(y), n, h4, w4, out_hw[0], out_hw[1], co, khp,
                                          stride[0], stride[1], _ws_code(*(tile or STEM_TILE)), N.ptr(s_sum),
                                          N.ptr(s_sq), slots, N.stream_ptr()), "conv_ws_stem")
    if keep_x4 is not None:
        keep_x4.append(x4)                    # the weight gradient reads the packed image again
    return y


def ws_depth_ok(k_total, d):
    """Load-ring depths the kernel instantiates for a reduction of ``k_total`` (csrc/conv_ws.hip
    dispatch_ws_d): K = 64 -> 2 or 4, K = 128 -> 4, longer K -> 3, 4 or 6 dividing K / 32."""
    ks = k_total // 32
    if ks == 2:
        return d in (2, 4)
    if ks == 3:
        return d == 3
    if ks == 4:
        return d == 4
    return ks > 4 and d in (3, 4, 6) and ks % d == 0


N.register("mdtf_conv3_rows", [N.P, N.P, N.P] + [N.I] * 4 + [N.P, N.P, N.I, N.P, N.P, N.P])
# row-staged 3x3 kernel (csrc/conv_rows.hip) for the 64 -> 64 channel, 56-wide stride-1 convolutions the
# weight-stationary table entries name; MDTF_CONV_ROWS=0 keeps the streamed kernel
CONV_ROWS = os.environ.get("MDTF_CONV_ROWS", "1") != "0"
DUAL_FUSED = [0]            # fused fan-out data gradients launched (tests)


def rows_ok(h_w, c, co, kh, kw, stride, pads, dil):
    """Shapes csrc/conv_rows.hip takes: 3x3, stride 1, pad 1, 64 -> 64 channels, 56 wide."""
    return (CONV_ROWS and c == 64 and co == 64 and kh == 3 and kw == 3 and tuple(stride) == (1, 1)
            and tuple(pads) == (1, 1, 1, 1) and tuple(dil) == (1, 1) and h_w[1] == 56)


def _ws_code(tp, nw, cg, d=4):
    """C-ABI tile code of csrc/conv_ws.hip: pixel subtiles, waves, channel groups, load-ring depth."""
    return tp + 10 * nw + 100 * cg + 1000 * d


def ws_fwd(x, wt, kh, kw, out_hw, stride, pads, dil, tile, stats=None, grid_cap=0, out=None):
    """Y = conv(X, W) on the weight-stationary kernel; ``wt`` = Wt[co][(kh,kw,ci)]
    (:func:`transpose_filter`).  ``tile`` = (tp, nw, cg[, d])."""
    n, h, wd, c = x.shape
    co = wt.shape[0]
    y = out if out is not None else torch.empty((n, out_hw[0], out_hw[1], co), dtype=x.dtype, device=x.device)
    s_sum, s_sq = stats if stats is not None else (None, None)
    slots = s_sum.shape[0] if s_sum is not None else 0
    if rows_ok((h, wd), c, co, kh, kw, stride, pads, dil) and tuple(out_hw) == (h, wd):
        N.check(N.fn("mdtf_conv3_rows")(N.ptr(x), N.ptr(wt), N.ptr(y), n, h, wd, 0, N.ptr(s_sum), N.ptr(s_sq), slots,
                                        N.ptr(None), N.ptr(None), N.stream_ptr()), "conv3_rows_fwd")
        return y
    N.check(N.fn("mdtf_conv_ws")(N.ptr(x), N.ptr(wt), N.ptr(y), n, h, wd, c, out_hw[0], out_hw[1], co, kh, kw,
                                 stride[0], stride[1], pads[0], pads[2], dil[0], dil[1], 0, _ws_code(*tile),
                                 int(grid_cap), N.ptr(s_sum), N.ptr(s_sq), slots, N.ptr(None), N.ptr(None),
                                 N.ptr(None), N.ptr(None), 0, 0, N.ptr(None), N.ptr(None), N.stream_ptr()),
            "conv_ws_fwd")
    return y


N.register("mdtf_conv_ws_bna", [N.P, N.P, N.P] + [N.I] * 7 + [N.P, N.P, N.I, N.P, N.P, N.P, N.P])


def bna_ok(ch, x_shape, w_shape, stride, pads, dil):
    """The forward of this conv can apply a pending BN + ReLU to its operand (``ops.bn`` ON_CONSUMER): the
    weight-stationary kernel on a 1x1 / stride-1 / unpadded conv with 64, 96 or 128 input channels."""
    kh, kw, ci, co = w_shape
    return (ch[0] == "ws" and kh == 1 and kw == 1 and tuple(stride) == (1, 1) and tuple(pads) == (0, 0, 0, 0)
            and tuple(dil) == (1, 1) and ci in (64, 96, 128) and ws_depth_ok(ci, ch[1][3] if len(ch[1]) > 3 else 4))


def ws_fwd_bna(x, wt, tile, stats, pend):
    """1x1 forward on the weight-stationary kernel whose operand is relu(x * scale + shift) of the pending BN
    ``pend = (a, x, scale|shift, mask)``: writes the BN output a and its mask as it goes (mdtf_conv_ws_bna)."""
    a, xin, ss, mask = pend
    n, h, wd, c = xin.shape
    co = wt.shape[0]
    y = torch.empty((n, h, wd, co), dtype=xin.dtype, device=xin.device)
    s_sum, s_sq = stats
    N.check(N.fn("mdtf_conv_ws_bna")(N.ptr(xin), N.ptr(wt), N.ptr(y), n, h, wd, c, co, _ws_code(*tile), 0,
                                     N.ptr(s_sum), N.ptr(s_sq), s_sum.shape[0], N.ptr(ss), N.ptr(a), N.ptr(mask),
                                     N.stream_ptr()), "conv_ws_bna")
    return y


def ws_dgrad(dy, w, x_shape, pads, dil, tile, out=None, accumulate=False, bn_stats=None, grid_cap=0, acc_src=None):
    """DX of a stride-1 conv on the weight-stationary kernel (the filter used flipped, HWIO as is).
    ``bn_stats = (x, relu_mask or None, psum, psq, slots)`` and ``acc_src`` as in :func:`mdtf_dgrad`."""
    n, h, wd, ci = x_shape
    kh, kw, _, co = w.shape
    dx = out if out is not None else torch.empty(x_shape, dtype=dy.dtype, device=dy.device)
    ph = (kh - 1) * dil[0] - pads[0]
    pw = (kw - 1) * dil[1] - pads[2]
    bx, bmask, bsum, bsq, bslots = bn_stats if bn_stats is not None else (None, None, None, None, 0)
    if (not accumulate and acc_src is None and rows_ok((h, wd), co, ci, kh, kw, (1, 1), pads, dil)
            and tuple(dy.shape[1:3]) == (h, wd)):
        N.check(N.fn("mdtf_conv3_rows")(N.ptr(dy), N.ptr(w), N.ptr(dx), n, h, wd, 1, N.ptr(bsum), N.ptr(bsq),
                                        int(bslots), N.ptr(bx), N.ptr(bmask), N.stream_ptr()), "conv3_rows_dgrad")
        return dx
    N.check(N.fn("mdtf_conv_ws")(N.ptr(dy), N.ptr(w), N.ptr(dx), n, dy.shape[1], dy.shape[2], co, h, wd, ci, kh, kw,
                                 1, 1, ph, pw, dil[0], dil[1], 1, _ws_code(*tile), int(grid_cap), N.ptr(None),
                                 N.ptr(None), 0, N.ptr(bx), N.ptr(bmask), N.ptr(bsum), N.ptr(bsq), int(bslots),
                                 int(bool(accumulate) or acc_src is not None),
                                 N.ptr(acc_src[0] if acc_src is not None else None),
                                 N.ptr(acc_src[1] if acc_src is not None else None), N.stream_ptr()), "conv_ws_dgrad")
    return dx


N.register("mdtf_conv_ws_dual", [N.P] * 5 + [N.I] * 10 + [N.P, N.P, N.P, N.P, N.I, N.P])
# fused fan-out data gradient (csrc/conv_ws.hip mdtf_conv_ws_dual) for a block input feeding a 1x1 / stride-1 conv
# and a strided 1x1 projection; MDTF_DUAL_DGRAD=0 runs the two data gradients one after the other
DUAL_DGRAD = os.environ.get("MDTF_DUAL_DGRAD", "1") != "0"
DUAL_TILE = tuple(int(v) for v in os.environ.get("MDTF_DUAL_TILE", "2,8,1").split(","))


def proj_deferrable(w_shape, stride, pads, dil):
    """A strided 1x1 projection whose data gradient may be deferred into the fused fan-out kernel."""
    return (DUAL_DGRAD and w_shape[0] == 1 and w_shape[1] == 1 and tuple(stride)[0] == tuple(stride)[1] > 1
            and tuple(pads) == (0, 0, 0, 0) and tuple(dil) == (1, 1) and w_shape[3] % 32 == 0)


def dual_ok(x_shape, w_shape, stride, pads, dil, pconv):
    """The completing 1x1 / stride-1 conv can run the deferred projection gradient ``pconv`` with its own."""
    if pconv is None or not (w_shape[0] == 1 and w_shape[1] == 1 and tuple(stride) == (1, 1)
                             and tuple(pads) == (0, 0, 0, 0) and tuple(dil) == (1, 1)):
        return False
    dy2, w2, s2 = pconv[:3]
    n, h, wd, c = x_shape
    c1, c2 = w_shape[3], w2.shape[3]
    return (c % 64 == 0 and c1 % 128 == 0 and c2 % 128 == 0 and 128 * (c1 + c2) <= 160 * 1024 and h > 1 and wd > 1
            and w2.shape[2] == c and tuple(s2) == (2, 2) and tuple(dy2.shape) == (n, -(-h // 2), -(-wd // 2), c2))


def ws_dual(dy, w, pconv, x_shape, tile=None, bn_stats=None):
    """DX = dgrad(dy, w) [1x1 / stride 1] + dgrad(dy2, w2) [1x1 / stride s2] in one pass (``pconv`` =
    (dy2, w2, stride)); ``bn_stats`` as in :func:`ws_dgrad`."""
    n, h, wd, c = x_shape
    dy2, w2, s2 = pconv[:3]
    dx = torch.empty(x_shape, dtype=dy.dtype, device=dy.device)
    bx, bmask, bsum, bsq, bslots = bn_stats if bn_stats is not None else (None, None, None, None, 0)
    tp, nw, cg = tile or DUAL_TILE
    if bn_stats is not None and tp > 2:
        tp = 2                                   # the BN-statistics epilogue's register budget
    N.check(N.fn("mdtf_conv_ws_dual")(N.ptr(dy), N.ptr(w), N.ptr(dy2), N.ptr(w2), N.ptr(dx), n, h, wd, c,
                                      w.shape[3], dy2.shape[1], dy2.shape[2], dy2.shape[3], s2[0],
                                      _ws_code(tp, nw, cg), N.ptr(bx), N.ptr(bmask), N.ptr(bsum), N.ptr(bsq),
                                      int(bslots), N.stream_ptr()), "conv_ws_dual")
    return dx


N.register("mdtf_conv_pp", [N.I, N.P, N.P, N.P] + [N.I] * 15 + [N.I, N.P, N.P, N.I, N.I] + [N.P] * 6 + [N.I, N.P])
PP_TILES = {0: (256, 256), 1: (256, 128), 2: (128, 256), 3: (128, 128), 4: (256, 192), 5: (128, 192)}


def pp_ok(pass_, c, co, stride, kh, kw, tile=None):
    """Shapes the ping-pong conv kernel (csrc/gemm_pp.hip mdtf_conv_pp) takes: the gathered channels are 64 * 2^p,
    <= 32 taps; dgrad stride 1 with Cin a multiple of the tile's columns."""
    g = c if pass_ == "fwd" else co
    if pass_ not in ("fwd", "dgrad") or g < 64 or g & (g - 1) or kh * kw > 32:
        return False
    if pass_ == "fwd":
        return co % 8 == 0
    return tuple(stride) == (1, 1) and (tile is None or c % PP_TILES[tile][1] == 0)


def pp_fwd(x, w, out_hw, stride, pads, dil, tile, stats=None, out=None):
    """Y = conv(X, W) on the ping-pong core (+ BN partials ``stats = (psum, psq)`` [slots][Cout])."""
    n = x.shape[0]
    co = w.shape[3]
    y = out if out is not None else torch.empty((n, out_hw[0], out_hw[1], co), dtype=x.dtype, device=x.device)
    s_sum, s_sq = stats if stats is not None else (None, None)
    slots = s_sum.shape[0] if s_sum is not None else 0
    N.check(N.fn("mdtf_conv_pp")(1, N.ptr(x), N.ptr(transpose_filter(w)), N.ptr(y), *_geo(x, w, out_hw, stride, pads, dil),
                                 int(tile), N.ptr(s_sum), N.ptr(s_sq), slots, 0, None, None, None, None, None, None, 0,
                                 N.stream_ptr()), "conv_pp_fwd")
    return y


def pp_dgrad(dy, w, x_shape, pads, dil, tile, out=None, accumulate=False, bn_stats=None, acc_src=None):
    """DX of a stride-1 conv on the ping-pong core; ``bn_stats`` / ``acc_src`` as in :func:`mdtf_dgrad`."""
    dx = out if out is not None else torch.empty(x_shape, dtype=dy.dtype, device=dy.device)
    n, h, wd, c = x_shape
    kh, kw, ci, co = w.shape
    geo = [n, h, wd, c, dy.shape[1], dy.shape[2], co, kh, kw, 1, 1, pads[0], pads[2], dil[0], dil[1]]
    bx, bmask, bsum, bsq, bslots = bn_stats if bn_stats is not None else (None, None, None, None, 0)
    ag, am = acc_src if acc_src is not None else (None, None)
    N.check(N.fn("mdtf_conv_pp")(2, N.ptr(dy), N.ptr(w), N.ptr(dx), *geo, int(tile), None, None, 0,
                                 int(bool(accumulate) or acc_src is not None), N.ptr(ag), N.ptr(am), N.ptr(bx),
                                 N.ptr(bmask), N.ptr(bsum), N.ptr(bsq), int(bslots), N.stream_ptr()), "conv_pp_dgrad")
    return dx


def mdtf_wgrad(x, dy, w_shape, stride, pads, dil, bm, bn, splits, out=None, ver=1, stages=2, store=False, fin=None):
    """fp32 HWIO weight gradient; accumulates into ``out`` when given (must be zeroed or a grad slot).  ``store``:
    the Variable whose grad slot ``out`` is -- when the launch reduces split-K slabs (v2 kernels), it claims the slot
    as the step's first writer and overwrites it (V.claim_store); the atomics epilogues accumulate (a claimed slot
    would need a zeroing launch of its own, which costs more than the fill that covers it).  ``fin``: (activation
    sink, statistics buffer, gamma, mean, invstd, M, C) of the BatchNorm whose backward finalize this launch runs
    in extra workgroups (v2 kernels; its result goes to the sink's ``early`` for ops.bn)."""
    dw = torch.zeros(w_shape, dtype=torch.float32, device=x.device) if out is None else out
    n, h, wd, c = x.shape
    kh, kw, ci, co = w_shape
    if ver in (2, 3):
        force = None
        if _SLAB_MODE not in ("0", "1"):          # MDTF_WGRAD_SLAB=0/1 pin it; else the table's per-shape choice
            ent = table().get(shape_key("wgrad", tuple(x.shape), tuple(w_shape), stride, pads, dil))
            if ent is not None and "slab" in ent:
                force = bool(ent["slab"])
        slab, cap = wgrad_slab(n * dy.shape[1] * dy.shape[2], kh * kw * ci, co, bm, bn, ver, int(splits), x.device,
                               force=force)
        if store is not False and store is not True:          # a Variable: claim only for the slab reduction
            var = store
            store = slab is not None and not WGRAD_INK and V.claim_store(var)
            if not store:
                V.note_accumulate(var)
        if store:
            N.fn("mdtf_set_wgrad_store")(1)
        if fin is not None:
            xs, sbuf, g, mean, invstd, M, C = fin
            fws = torch.empty(5 * C, dtype=torch.float32, device=x.device)
            N.check(N.fn("mdtf_set_wgrad_fin")(N.ptr(sbuf[0]), N.ptr(sbuf[1]), int(sbuf.shape[1]), N.ptr(g),
                                               N.ptr(mean), N.ptr(invstd), N.ptr(fws), int(M), int(C)), "wgrad_fin")
        try:
            with slab_side(slab if out is not None else None), wgrad_tickets(slab):
                N.check(N.fn("mdtf_conv_wgrad_v2")(N.ptr(x), N.ptr(dy), N.ptr(dw), n, h, wd, c, dy.shape[1],
                                                   dy.shape[2], co, kh, kw, stride[0], stride[1], pads[0], pads[2],
                                                   dil[0], dil[1], _v2_code(bm, stages, ver), bn, int(splits),
                                                   N.ptr(slab), cap, N.stream_ptr()), "conv_wgrad_v2")
        finally:
            if store:
                N.fn("mdtf_set_wgrad_store")(0)
            if fin is not None:
                N.fn("mdtf_set_wgrad_fin")(None, None, 0, None, None, None, None, 0, 0)   # (consumed or cancelled)
        if fin is not None:
            xs.early = (fws, None)
        return dw
    N.check(N.fn("mdtf_conv_wgrad")(N.ptr(x), N.ptr(dy), N.ptr(dw), n, h, wd, c, dy.shape[1], dy.shape[2], co, kh,
                                    kw, stride[0], stride[1], pads[0], pads[2], dil[0], dil[1], bm, bn, int(splits),
                                    N.stream_ptr()), "conv_wgrad")
    return dw


def _pads_ok(pads):
    # the kernels take (top, left) padding; bottom/right are implied by the output size
    return True


BWD_STATS = os.environ.get("MDTF_BN_BWD_STATS", "1") != "0"   # BN backward statistics from the dgrad epilogue
STAT_SLOTS = 64   # atomic partial rows of the fused BN statistics (csrc/conv_igemm.hip kStatSlots)
MAX_STAT_SLOTS = int(os.environ.get("MDTF_BN_MAX_SLOTS", "128"))   # cap of the adaptive slot count (A/B: 128 beat 1024 by 0.4%)
_STATS = {}       # device -> [flat fp32 buffer, dirty]: persistent, re-zeroed by the BN finalize kernel


def _stats_buffer(co, device, slots=STAT_SLOTS):
    """Zeroed [2, STAT_SLOTS, co] partial-sum buffer for a conv epilogue.

    One persistent buffer per device: the following BatchNorm's finalize
    kernel reads and re-zeroes it (``bn_fwd_stats``), so no fill kernel runs per
    conv.  If a previous conv's statistics were never consumed, zero it here.
    """
    ent = _STATS.get(device)
    need = 2 * slots * co
    if ent is None or ent[0].numel() < need:
        ent = [torch.zeros(max(need, 2 * STAT_SLOTS * 2048), dtype=torch.float32, device=device), False]
        _STATS[device] = ent
    if ent[1]:
        ent[0].zero_()
    ent[1] = True
    return ent[0][:need].view(2, slots, co)


def stats_consumed(device):
    ent = _STATS.get(device)
    if ent is not None:
        ent[1] = False


def stat_slots(mtiles):
    """Atomic partial rows for epilogue statistics: one per M tile in deterministic mode,
    else ~8 M tiles per row (64..MAX_STAT_SLOTS rows): low contention, small finalize."""
    if N.deterministic():
        return mtiles
    slots = STAT_SLOTS
    while slots < MAX_STAT_SLOTS and slots * 8 < mtiles:
        slots *= 2
    return slots


# Weight gradients on a side stream: a conv's wgrad does not feed the rest of backward (only the flat
# gradient buffer), so it runs on its own HIP stream beside the dgrad -> BN-backward chain and fills
# the CUs that chain's memory-bound and small kernels leave idle.  Captured hipGraphs keep the two
# streams as concurrent branches.  The gradient buffer is read only after join_side_streams()
# (bucket all-reduce launch, end of backward).  Measured on ResNet-50 (scripts/gpu.sh envab): -0.3 %
# (the chain's kernels already keep HBM busy), so it is opt-in: MDTF_WGRAD_STREAM=1.
WGRAD_STREAM = os.environ.get("MDTF_WGRAD_STREAM", "0") == "1"
_SIDE = {}        # device -> side stream
_PENDING = set()  # devices with side-stream work the main stream has not joined yet


def _side_stream(device):
    s = _SIDE.get(device)
    if s is None:
        s = torch.cuda.Stream(device=device)
        _SIDE[device] = s
    return s


# Split-K slab reductions of weight gradients on the side stream (MDTF_SLAB_SIDE=1): the wgrad kernel stays in
# line, only its reduction pass (10 us per ResNet-50 conv, 36 per step) forks off the dgrad -> BN-backward chain
# into the gradient buffer, joined by join_side_streams() like the side-stream weight gradients above.
SLAB_SIDE = os.environ.get("MDTF_SLAB_SIDE", "0") == "1"


class slab_side:
    """Context for one native launch whose partial-sum reduction (a weight gradient's split-K slab, a LayerNorm's
    gamma / beta block partials in ``ws``) goes to the side stream; ``setter`` names the native stream hook."""

    def __init__(self, slab, setter="mdtf_set_slab_stream"):
        self.slab = slab if (SLAB_SIDE and slab is not None and slab.is_cuda) else None
        self.setter = setter

    def __enter__(self):
        if self.slab is not None:
            self.side = _side_stream(self.slab.device)
            N.fn(self.setter)(ctypes.c_void_p(self.side.cuda_stream))
        return self

    def __exit__(self, *exc):
        if self.slab is not None:
            N.fn(self.setter)(None)
            self.slab.record_stream(self.side)      # read by the side stream's reduction
            _PENDING.add(self.slab.device)
        return False


def join_side_streams():
    """Make the current stream wait for every weight gradient issued on the side streams."""
    for dev in list(_PENDING):
        torch.cuda.current_stream(dev).wait_stream(_SIDE[dev])
    _PENDING.clear()


_BSTATS = {}      # (device, C, slots) -> free zeroed [2, slots, C] buffers (BN backward statistics)


def bwd_stats_acquire(device, C, slots):
    pool = _BSTATS.setdefault((device, C, slots), [])
    return pool.pop() if pool else torch.zeros((2, slots, C), dtype=torch.float32, device=device)


def _early_finalize(xs, sbuf):
    """The BN whose output gradient this data gradient just completed may finalize its backward statistics now, on
    a side stream beside this conv's weight gradient (``ops.bn`` EARLY_FIN), instead of after it.  Returns the
    arguments of a finalize that can ride on this conv's weight-gradient launch instead (``ops.bn`` WG_FIN) or
    None."""
    req = xs.stat_req
    if req is not None and len(req) > 2 and req[2] is not None:
        xs.early = req[2](sbuf)
        return None
    if req is not None and len(req) > 3 and req[3] is not None:
        return (xs, sbuf) + tuple(req[3])
    return None


def bwd_stats_release(buf, zeroed):
    """Return a buffer to the pool; ``zeroed``: the BN finalize already re-zeroed it."""
    if not zeroed:
        buf.zero_()
    _BSTATS.setdefault((buf.device, buf.shape[2], buf.shape[1]), []).append(buf)


class _Conv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, stride, pads, dil, out_hw, want_stats):
        from . import actsink
        ctx.set_materialize_grads(False)      # no zero-filled grads for the (non-differentiable) stats outputs
        ctx.x_sink = actsink.sink_of(x)       # fanned-out input: dgrad accumulates into the producer's sink
        if ctx.x_sink is not None:
            ctx.x_sink.register()
        from . import bn as _bn
        pend = _bn.take_pending(x)             # x: a BN output its producer left for this conv to apply
        x = x.contiguous()
        w = w.contiguous()
        ch = choose("fwd", x.shape, w.shape, stride, pads, dil)
        if pend is not None and not (want_stats and bna_ok(ch, x.shape, w.shape, stride, pads, dil)):
            _bn.apply_pending(pend)
            pend = None
        stats = None
        # want_stats 2: a private zeroed partial buffer (statistics consumed later than the next conv, e.g. a
        # deferred shortcut BN), else the persistent per-device one
        sbuf = _stats_buffer if want_stats != 2 else (
            lambda co, dev, slots=STAT_SLOTS: torch.zeros((2, slots, co), dtype=torch.float32, device=dev))
        if ch[0] == "mdtf":
            if want_stats:
                co = w.shape[3]
                slots = stat_slots(-(-x.shape[0] * out_hw[0] * out_hw[1] // ch[1]))
                buf = sbuf(co, x.device, slots)
                stats = (buf[0], buf[1])
            y = mdtf_fwd(x, w, out_hw, stride, pads, dil, ch[1], ch[2], stats, ch[4], ch[5])
        elif ch[0] == "pp":
            if want_stats:
                co = w.shape[3]
                slots = stat_slots(-(-x.shape[0] * out_hw[0] * out_hw[1] // PP_TILES[ch[1]][0]))
                buf = sbuf(co, x.device, slots)
                stats = (buf[0], buf[1])
            y = pp_fwd(x, w, out_hw, stride, pads, dil, ch[1], stats)
        elif ch[0] == "stem":
            if want_stats:
                buf = sbuf(w.shape[3], x.device, STAT_SLOTS)
                stats = (buf[0], buf[1])
            keep = []
            y = stem_fwd(x, w, out_hw, stride, pads, stats, keep_x4=keep)
            ctx.stem_x4 = keep[0]
        elif ch[0] == "ws":
            if want_stats:
                buf = sbuf(w.shape[3], x.device, STAT_SLOTS)
                stats = (buf[0], buf[1])
            if pend is not None:
                y = ws_fwd_bna(x, transpose_filter(w), ch[1], stats, pend)
                _bn.ON_CONSUMER_USED[0] += 1
            else:
                y = ws_fwd(x, transpose_filter(w), w.shape[0], w.shape[1], out_hw, stride, pads, dil, ch[1], stats)
        elif ch[0] == "winograd":
            y = winograd.winograd_fwd(x, w, out_hw, pads)
        else:
            y = miopen_fwd(x, w, stride, pads, dil)
        ctx.save_for_backward(x, w)
        ctx.args = (stride, pads, dil)
        ctx.w_dtype = w.dtype
        ctx.sink = V.grad_sink(w)
        if want_stats:
            if stats is None:
                empty = torch.empty(0, device=x.device)
                ctx.mark_non_differentiable(empty, empty)
                return y, empty, empty
            ctx.mark_non_differentiable(stats[0], stats[1])
            return y, stats[0], stats[1]
        return y

    @staticmethod
    def backward(ctx, dy, *unused):
        x, w = ctx.saved_tensors
        if dy is None:
            return None, None, None, None, None, None, None
        stride, pads, dil = ctx.args
        dy = dy.contiguous()
        need_dx, need_dw = ctx.needs_input_grad[0], ctx.needs_input_grad[1]
        fin_job = None        # a BN backward finalize this conv's weight-gradient launch may run (ops.bn WG_FIN)
        dx = dw = None
        cd = choose("dgrad", x.shape, w.shape, stride, pads, dil) if need_dx else None
        cw = choose("wgrad", x.shape, w.shape, stride, pads, dil) if need_dw else None
        if need_dw and cw[0] == "stem" and getattr(ctx, "stem_x4", None) is None:
            cw = ("miopen",)                   # the forward did not leave the packed image
        lib_dx = need_dx and cd[0] in ("miopen", "stem")
        lib_dw = need_dw and cw[0] == "miopen"
        sink = ctx.sink
        if lib_dx or lib_dw:
            ldx, ldw = miopen_bwd(x, w, dy, stride, pads, dil, lib_dx, lib_dw)
            if lib_dx:
                dx = ldx
            if lib_dw:
                if sink is not None:
                    sink.grad.add_(ldw)            # straight into the fp32 grad slot
                    dw = V.grad_marker(w)
                else:
                    dw = ldw
        xs = ctx.x_sink if need_dx else None
        if (xs is not None and not lib_dx and xs.idle() and not xs.completing()
                and proj_deferrable(w.shape, stride, pads, dil) and cd[0] in ("mdtf", "pp")
                and (cd[0] == "pp" or cd[4] in (2, 3))):
            # strided 1x1 projection, first contributor: leave its data gradient to the block's 1x1 conv
            def _run(out, acc, dy=dy, w=w, xshape=tuple(x.shape), stride=stride, pads=pads, dil=dil, cd=cd):
                if cd[0] == "pp":
                    return pp_dgrad(dy, w, xshape, pads, dil, cd[1], out=out, accumulate=acc)
                return mdtf_dgrad(dy, w, xshape, stride, pads, dil, cd[1], cd[2], cd[4], cd[5], out=out,
                                  accumulate=acc)
            xs.defer_conv(dy, w, tuple(stride), _run)
            need_dx = False
        elif xs is not None and not lib_dx and dual_ok(x.shape, w.shape, stride, pads, dil, xs.pconv) \
                and xs.buf is None and xs.pend is None:
            pc = xs.take_conv()
            bst = None
            if xs.stat_req is not None and xs.completing() and BWD_STATS and not N.deterministic():
                bx, bmask = xs.stat_req[:2]
                sbuf = bwd_stats_acquire(x.device, x.shape[3], STAT_SLOTS)
                bst = (bx, bmask, sbuf[0], sbuf[1], sbuf.shape[1])
            xs.written(ws_dual(dy, w, pc, x.shape, bn_stats=bst))
            if bst is not None:
                xs.stats = sbuf
                fin_job = _early_finalize(xs, sbuf)
            DUAL_FUSED[0] += 1
            need_dx = False
        if need_dx and cd[0] == "winograd":
            dx = winograd.winograd_dgrad(dy, w, x.shape, pads)
        elif need_dx and cd[0] == "ws":
            tile = cd[1]
            if xs is not None:
                buf, acc, pend = xs.target_ex()
                bst = None
                if xs.stat_req is not None and xs.completing() and BWD_STATS:
                    bx, bmask = xs.stat_req[:2]
                    sbuf = bwd_stats_acquire(x.device, x.shape[3], STAT_SLOTS)
                    bst = (bx, bmask, sbuf[0], sbuf[1], sbuf.shape[1])
                    tile = (2,) + tuple(tile[1:])      # the statistics epilogue's register budget
                xs.written(ws_dgrad(dy, w, x.shape, pads, dil, tile, out=buf, accumulate=acc, bn_stats=bst,
                                    acc_src=pend))
                if bst is not None:
                    xs.stats = sbuf
                    fin_job = _early_finalize(xs, sbuf)
            else:
                dx = ws_dgrad(dy, w, x.shape, pads, dil, tile)
        elif need_dx and cd[0] == "pp":
            if xs is not None:
                buf, acc, pend = xs.target_ex()
                bst = None
                if xs.stat_req is not None and xs.completing() and BWD_STATS and not N.deterministic():
                    bx, bmask = xs.stat_req[:2]
                    sbuf = bwd_stats_acquire(x.device, x.shape[3],
                                             stat_slots(-(-x.numel() // x.shape[3] // PP_TILES[cd[1]][0])))
                    bst = (bx, bmask, sbuf[0], sbuf[1], sbuf.shape[1])
                xs.written(pp_dgrad(dy, w, x.shape, pads, dil, cd[1], out=buf, accumulate=acc, bn_stats=bst,
                                    acc_src=pend))
                if bst is not None:
                    xs.stats = sbuf
                    fin_job = _early_finalize(xs, sbuf)
            else:
                dx = pp_dgrad(dy, w, x.shape, pads, dil, cd[1])
        elif need_dx and not lib_dx:
            if xs is not None and cd[4] in (2, 3):
                buf, acc, pend = xs.target_ex()
                bst = None
                if xs.stat_req is not None and xs.completing() and BWD_STATS and not N.deterministic():
                    # this dgrad completes the BN output's gradient: emit the BN backward statistics
                    bx, bmask = xs.stat_req[:2]
                    sbuf = bwd_stats_acquire(x.device, x.shape[3], stat_slots(-(-x.numel() // x.shape[3] // cd[1])))
                    bst = (bx, bmask, sbuf[0], sbuf[1], sbuf.shape[1])
                xs.written(mdtf_dgrad(dy, w, x.shape, stride, pads, dil, cd[1], cd[2], cd[4], cd[5], out=buf,
                                      accumulate=acc, bn_stats=bst, acc_src=pend))
                if bst is not None:
                    xs.stats = sbuf
                    fin_job = _early_finalize(xs, sbuf)
                dx = None
            else:
                dx = mdtf_dgrad(dy, w, x.shape, stride, pads, dil, cd[1], cd[2], cd[4], cd[5])
        if xs is not None and dx is not None:
            xs.adopt_or_add(dx)                    # library / v1 dgrad: contribute the tensor
            dx = None
        if need_dw and cw[0] == "stem":
            if sink is not None:
                stem_wgrad(ctx.stem_x4, dy, w.shape, stride, out=sink.grad)
                dw = V.grad_marker(w)
            else:
                dw = stem_wgrad(ctx.stem_x4, dy, w.shape, stride)
                if dw.dtype != ctx.w_dtype:
                    dw = dw.to(ctx.w_dtype)
            ctx.stem_x4 = None
        elif need_dw and not lib_dw:
            if sink is not None:
                # fp32 atomics of the wgrad kernel accumulate into the flat gradient buffer
                if WGRAD_STREAM and x.is_cuda:
                    V.note_accumulate(sink)           # (zeroes a store-first slot the fill skipped)
                    side = _side_stream(x.device)
                    side.wait_stream(torch.cuda.current_stream(x.device))
                    with torch.cuda.stream(side):
                        mdtf_wgrad(x, dy, w.shape, stride, pads, dil, cw[1], cw[2], cw[3], out=sink.grad,
                                   ver=cw[4], stages=cw[5])
                    x.record_stream(side)
                    dy.record_stream(side)
                    _PENDING.add(x.device)
                else:
                    # v2 kernels with a split-K slab overwrite the slot as the step's first writer of it
                    # (V.claim_store): no zero fill, no read of the slot in the slab reduction
                    if cw[4] not in (2, 3):
                        V.note_accumulate(sink)
                    mdtf_wgrad(x, dy, w.shape, stride, pads, dil, cw[1], cw[2], cw[3], out=sink.grad, ver=cw[4],
                               stages=cw[5], store=sink if cw[4] in (2, 3) else False,
                               fin=fin_job if cw[4] in (2, 3) else None)
                    fin_job = None
                dw = V.grad_marker(w)
            else:
                dw = mdtf_wgrad(x, dy, w.shape, stride, pads, dil, cw[1], cw[2], cw[3], ver=cw[4], stages=cw[5])
                if dw.dtype != ctx.w_dtype:
                    dw = dw.to(ctx.w_dtype)
        return dx, dw, None, None, None, None, None


def _out_hw(x, w, stride, pads, dil):
    n, h, wd, c = x.shape
    kh, kw, _, co = w.shape
    oh = (h + pads[0] + pads[1] - ((kh - 1) * dil[0] + 1)) // stride[0] + 1
    ow = (wd + pads[2] + pads[3] - ((kw - 1) * dil[1] + 1)) // stride[1] + 1
    return oh, ow


def conv2d_nhwc(x, w, stride, pads, dil, bias=None, act=None):
    if x.dtype != torch.bfloat16:
        raise TypeError("mdtf conv kernels take bf16 activations, got %s" % x.dtype)
    if w.dtype != x.dtype:
        w = w.to(x.dtype)
    y = _Conv.apply(x, w, tuple(stride), tuple(pads), tuple(dil), _out_hw(x, w, stride, pads, dil), False)
    if bias is not None or act is not None:
        from . import kernels
        y = kernels.bias_act(y, bias, act)
    return y


def conv2d_stats_nhwc(x, w, stride, pads, dil, private=False):
    """conv2d that also returns fused BN statistics partials ``(psum, psq, P)`` (or None); ``private``: in a
    buffer of their own (consumed after later convs have run) instead of the shared per-device one."""
    if x.dtype != torch.bfloat16:
        raise TypeError("mdtf conv kernels take bf16 activations, got %s" % x.dtype)
    if w.dtype != x.dtype:
        w = w.to(x.dtype)
    y, psum, psq = _Conv.apply(x, w, tuple(stride), tuple(pads), tuple(dil), _out_hw(x, w, stride, pads, dil),
                               2 if private else True)
    if psum.numel() == 0:
        return y, None
    return y, (psum, psq, psum.shape[0])


def conv2d_dgrad_nhwc(x, w, out_shape, stride, pads):
    """conv2d_transpose == data-gradient of conv2d with filter [kh, kw, cout_op, cin_op]."""
    n, oh, ow, co = out_shape
    kh, kw, wco, wci = w.shape
    wb = w.to(x.dtype).contiguous()
    ch = choose("dgrad", (n, oh, ow, co), (kh, kw, co, wci), stride, pads, (1, 1))
    if ch[0] == "mdtf":
        return _ConvT.apply(x, wb, tuple(stride), tuple(pads), (n, oh, ow, co), ch[1], ch[2], ch[4], ch[5])
    xc = x.permute(0, 3, 1, 2)
    wt = w.permute(3, 2, 0, 1).to(x.dtype)
    y = F.conv_transpose2d(xc, wt, None, stride, 0)
    y = y[:, :, pads[0]:pads[0] + oh, pads[2]:pads[2] + ow]
    if y.shape[2] < oh or y.shape[3] < ow:
        y = F.pad(y, (0, ow - y.shape[3], 0, oh - y.shape[2]))
    return y.permute(0, 2, 3, 1).contiguous()


class _ConvT(torch.autograd.Function):
    """Transposed conv as conv dgrad (fwd) with conv fwd / wgrad for its backward."""

    @staticmethod
    def forward(ctx, x, w, stride, pads, out_shape, bm, bn, ver, stages):
        x = x.contiguous()
        y = mdtf_dgrad(x, w, out_shape, stride, pads, (1, 1), bm, bn, ver, stages)
        ctx.save_for_backward(x, w)
        ctx.args = (stride, pads)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        stride, pads = ctx.args
        dy = dy.contiguous()
        oh, ow = x.shape[1], x.shape[2]
        bm, bn = _default_tile(w.shape[3])
        dx = mdtf_fwd(dy, w, (oh, ow), stride, pads, (1, 1), bm, bn) if ctx.needs_input_grad[0] else None
        dw = None
        if ctx.needs_input_grad[1]:
            dw = mdtf_wgrad(dy, x, w.shape, stride, pads, (1, 1), 128 if w.shape[0] * w.shape[1] * w.shape[2] >= 128
                            else 64, 128 if w.shape[3] % 128 == 0 else 64, 0)
        return dx, dw, None, None, None, None, None, None, None
