"""The ping-pong MFMA GEMM core (``csrc/gemm_pp.hip``) as torch-facing calls.

Three layouts cover every dense-layer product without a transposed or concatenated copy of anything:

* ``fwd``   ``y = act(x @ [w_0|..] + [b_0|..])``   x [M, K], w_s [K, Ns]        (layout 0)
* ``dgrad`` ``dx (+)= dy @ [w_0|..]^T``             dy [M, sum Ns], w_s [K, Ns]  (layout 1)
* ``wgrad`` ``g_s += x^T @ dy[:, seg s]`` (fp32)    x [M, K], dy [M, sum Ns]     (layout 2)

Several weight matrices that share an input (BERT's q|k|v) are *segments* of one launch: the kernel picks the
segment per LDS unit (forward: output columns; data gradient: the reduction), so there is no ``torch.cat`` of
the weights in either direction and the weight gradient lands directly in each variable's fp32 slot.

Tile codes: 0 = 256x256, 1 = 256x128, 2 = 128x256, 3 = 128x128, 4 = 256x192, 5 = 128x192 (rows x cols of C).
``pick_tile`` models the grid's wave quantisation on the 256 CUs and the per-tile efficiency of each shape;
``TILES`` pins measured per-shape choices (``bench/gemm_pp_probe.py`` on an MI355X).
"""
import ctypes
import os

import torch

from . import _native as N

N.register("mdtf_gemm_pp", [N.P, N.L, N.P, N.L, N.I, N.I, N.I, N.I, N.I, N.I, N.I, N.I, N.P, N.L, N.P, N.P, N.I,
                            N.I, N.P, N.I, N.P, N.L, N.P, N.P])

_TILE_DIMS = {0: (256, 256), 1: (256, 128), 2: (128, 256), 3: (128, 128), 4: (256, 192), 5: (128, 192)}
# relative time per unit of tile work (LDS / L2 bytes per FLOP grow as the tile shrinks), from the probe
_TILE_COST = {0: 1.0, 1: 1.14, 2: 1.10, 3: 1.35, 4: 1.05, 5: 1.16}
CUS = 256

# (layout, M, N, K) -> (tile, splits): measured choices (graph-timed on MI355X, bench/gemm_pp_probe.py); MDTF_PP_TILES
# "layout,M,N,K:tile,splits;..." pins more (in-step A/B)
TILES = {}
for _ent in filter(None, os.environ.get("MDTF_PP_TILES", "").split(";")):
    _k, _v = _ent.split(":")
    TILES[tuple(int(t) for t in _k.split(","))] = tuple(int(t) for t in _v.split(","))

ACT = {None: 0, "relu": 1, "gelu": 2}


def _valid(layout, tile, M, Nn):
    bm, bn = _TILE_DIMS[tile]
    if layout == 2 and M % bm:          # transposed A must not straddle its edge
        return False
    if layout in (0, 2) and Nn % bn:    # transposed B
        return False
    return True


def pick_tile(layout, M, Nn, K, seg_cols=None):
    """(tile, splits) for C[M][Nn] with reduction K (layout 2 may split K)."""
    t = TILES.get((layout, M, Nn, K))
    if t is not None:
        return t
    best = None
    for tile in _TILE_DIMS:
        bm, bn = _TILE_DIMS[tile]
        if not _valid(layout, tile, M, Nn):
            continue
        if seg_cols and layout in (0, 2) and seg_cols % bn:
            continue
        ntiles = -(-M // bm) * -(-Nn // bn)
        for sp in ((1,) if layout != 2 else (1, 2, 3, 4, 6, 8)):
            if sp > 1 and K // 64 < sp * 8:
                continue
            nt = ntiles * sp
            rounds = -(-nt // CUS)
            per = (bm * bn) / 65536.0 * (K / 64.0 / sp + 3.0) * _TILE_COST[tile]    # +3: pipeline fill / epilogue
            cost = rounds * per + (0.4 * (bm * bn) / 65536.0 * sp if sp > 1 else 0.0)  # split-K atomics
            if best is None or cost < best[0]:
                best = (cost, tile, sp)
    if best is None:
        return None
    return best[1], best[2]


def _arr(ts):
    a = (ctypes.c_void_p * 4)()
    for i, t in enumerate(ts):
        a[i] = t if isinstance(t, int) else (t.data_ptr() if t is not None else 0)
    return a


def _call(A, lda, bsegs, ldb, M, Nn, K, layout, tile, splits, seg_cols, C=None, ldc=0, biases=None, pre=None,
          act=0, accumulate=0, act_pre=None, act_bwd=0, cfs=None, ldcf=0, dbs=None):
    return N.fn("mdtf_gemm_pp")(
        N.ptr(A), lda, ctypes.cast(_arr(bsegs), ctypes.c_void_p), ldb, M, Nn, K, layout, tile, splits, len(bsegs),
        seg_cols, N.ptr(C), ldc, ctypes.cast(_arr(biases), ctypes.c_void_p) if biases else None, N.ptr(pre), act,
        accumulate, N.ptr(act_pre), act_bwd, ctypes.cast(_arr(cfs), ctypes.c_void_p) if cfs else None, ldcf,
        ctypes.cast(_arr(dbs), ctypes.c_void_p) if dbs else None, N.stream_ptr())


def fwd(x, ws, biases=None, act=0, pre=None, out=None, tile=None):
    """act(x @ [ws...] + [biases...]) in bf16.  x [M, K] (unit column stride); ws: one [K, N] or a list of
    equal [K, Ns] segments (contiguous); biases: matching bf16 vectors or None; pre: the bf16 pre-activation
    output (act != 0).  Returns None when the kernel does not take the shape."""
    ws = ws if isinstance(ws, (list, tuple)) else [ws]
    M, K = x.shape
    ns = ws[0].shape[1]
    Nn = ns * len(ws)
    if tile is None and os.environ.get("MDTF_PP_FWD_TILE"):        # (A/B switch: force the forward tile code)
        tile = int(os.environ["MDTF_PP_FWD_TILE"])
    t = (tile, 1) if tile is not None else pick_tile(0, M, Nn, K, ns if len(ws) > 1 else None)
    if t is None:
        return None
    y = out if out is not None else torch.empty((M, Nn), dtype=x.dtype, device=x.device)
    rc = _call(x, x.stride(0), ws, ws[0].stride(0), M, Nn, K, 0, t[0], 1, ns, C=y, ldc=y.stride(0),
               biases=biases if biases and biases[0] is not None else None, pre=pre, act=act)
    if rc == -2:
        return None
    N.check(rc, "gemm_pp fwd")
    return y


def dgrad(dy, ws, out=None, accumulate=False, act_pre=None, act_bwd=0, tile=None):
    """dy @ [ws...]^T -> [M, K] bf16 (dy [M, sum Ns]; ws [K, Ns] segments).  ``accumulate``: out += ...;
    ``act_pre``/``act_bwd``: multiply by the producer's activation derivative at ``act_pre`` [M, K]."""
    ws = ws if isinstance(ws, (list, tuple)) else [ws]
    M, Nn = dy.shape
    K = ws[0].shape[0]
    t = (tile, 1) if tile is not None else pick_tile(1, M, K, Nn)
    if t is None:
        return None
    dx = out if out is not None else torch.empty((M, K), dtype=dy.dtype, device=dy.device)
    rc = _call(dy, dy.stride(0), ws, ws[0].stride(0), M, K, Nn, 1, t[0], 1, ws[0].shape[1], C=dx, ldc=dx.stride(0),
               accumulate=int(accumulate), act_pre=act_pre, act_bwd=act_bwd)
    if rc == -2:
        return None
    N.check(rc, "gemm_pp dgrad")
    return dx


def wgrad_into(gws, x, dy, dbs=None, tile=None, splits=None):
    """gws[s] [K, Ns] fp32 += x^T @ dy[:, segment s] (x [M, K], dy [M, sum Ns] bf16, unit column strides);
    ``dbs``: fp32 [Ns] slots that also receive the column sums of dy (the bias gradients).  False when the
    kernel does not take the shape (the caller falls back)."""
    gws = gws if isinstance(gws, (list, tuple)) else [gws]
    M, K = x.shape
    Nn = dy.shape[1]
    ns = gws[0].shape[1]
    if tile is None:
        t = pick_tile(2, K, Nn, M, ns if len(gws) > 1 else None)
        if t is None:
            return False
        tile, sp = t
        splits = splits or sp
    bsegs = [dy.data_ptr() + 2 * ns * i for i in range(len(gws))]     # dy's column segments, row stride = Nn
    rc = _call(x, x.stride(0), bsegs, dy.stride(0), K, Nn, M, 2, tile, splits or 1, ns, cfs=gws,
               ldcf=gws[0].stride(0), dbs=dbs)
    if rc == -2:
        return False
    N.check(rc, "gemm_pp wgrad")
    return True


# ---------------------------------------------------------------------------------------------------------------
# Weight-gradient kernel (csrc/gemm_wg.hip): C_s (fp32) += x^T dy[:, seg s], both operands k-major, split-K
# partials reduced by the last arriving workgroup of each tile (no fp32 atomics on C, deterministic order).
N.register("mdtf_gemm_wg", [N.P, N.L, N.P, N.L, N.I, N.I, N.I, N.I, N.I, N.P, N.L, N.P, N.I, N.I, N.I, N.P, N.P,
                            N.I, N.P])
N.register("mdtf_gemm_wg_slab_floats", [N.I, N.I, N.I, N.I], N.L)
N.register("mdtf_gemm_wg_slab_floats_k", [N.I, N.I, N.I, N.I, N.I], N.L)
# stream-K weight gradients (MDTF_WG_SK=1): every CU runs the same number of K-tiles, cut at tile boundaries,
# instead of tiles x splits workgroups that leave CUs idle (BERT-base: 72 tiles x 3 = 216 of 256 CUs).  Off: a
# worker whose range crosses a tile boundary pays a second pipeline fill + slab epilogue (+ the last arriver's
# sum) on the critical path -- 256 workers 72-86 us vs 55-64 us for the split grid (profiles/wg_sk_probe_r5w.jsonl),
# BERT step 6045 vs 6509 seq/s
WG_SK = os.environ.get("MDTF_WG_SK", "0") == "1"

# (M, N, K) -> (bm, stages, splits): graph-timed on an MI355X (bench/gemm_wg_probe.py, profiles/gemm_wg_probe_r3b.jsonl;
# the 3/4-stage rings and the mid-tile-barrier loop (stages < 0) measured slower than the 2-stage ring on every shape)
# In the BERT-base step the 256-row kernels gain from the third ring stage (HBM-cold saved activations; graph-timed
# with MALL-resident operands 2 and 3 stages tie): MDTF_WG_STAGES=3 vs 2, alternating: 6485 / 6530 vs 6378 / 6420 seq/s
# (FFN-out 3072 x 768: 256-row 3-stage 6368 / 6362 vs 128-row 2-stage 6356 / 6336 seq/s)
# Round 6 (write-through slab publish + store-first slots): in-step re-tune moved the q|k|v and FFN-out shapes to
# two 128-row workgroups per CU (bench/bert_wg_tune.py, profiles/bert_wg_tune_r6f.md: step 9.511 -> 9.402 ms); the
# final-tree re-tune moved the FFN-in shape too (bert_wg_tune_r6w.md; captured A/B 7049 vs 7024 seq/s, 6 of 6 pairs)
WG_TILES = {(768, 2304, 8192): (128, 2, 4), (768, 3072, 8192): (128, 2, 3), (3072, 768, 8192): (128, 2, 3),
            (768, 768, 8192): (128, 2, 6), (1024, 3072, 8192): (256, 3, 2), (1024, 4096, 8192): (256, 3, 2),
            (4096, 1024, 8192): (256, 3, 2)}
# MDTF_WG_TILES="M,N,K:bm,stages,splits;...": override entries (in-step A/B of a tuner's proposal)
for _ent in filter(None, os.environ.get("MDTF_WG_TILES", "").split(";")):
    _k, _v = _ent.split(":")
    WG_TILES[tuple(int(t) for t in _k.split(","))] = tuple(int(t) for t in _v.split(","))
_TICKETS = {}
# MDTF_WG_STAGES: force the ring depth of the table entries (in-step A/B: the operands of the step are HBM-cold,
# the graph-timed probe's are MALL-resident)
_WG_STAGES = int(os.environ["MDTF_WG_STAGES"]) if os.environ.get("MDTF_WG_STAGES") else None


def _tickets(device, n):
    """Zeroed per-tile arrival tickets, one buffer per (device, stream): launches on one stream are ordered, and
    every launch leaves its tickets at zero (the last arriver resets them)."""
    key = (str(device), torch.cuda.current_stream(device).cuda_stream)
    t = _TICKETS.get(key)
    if t is None or t.numel() < n:
        t = torch.zeros(max(n, 4096), dtype=torch.int32, device=device)
        _TICKETS[key] = t
    return t


def wg_pick(M, Nn, K):
    """(bm, stages, splits) for C[M][Nn] += over K tokens.  Measured: one 256-row workgroup per CU with a
    3-stage ring (in the step) beats the 128-row pairs; split until the tiles x splits grid just fills the 256 CUs (a second
    round of workgroups costs more than it saves), keeping >= 16 K-tiles per split."""
    t = WG_TILES.get((M, Nn, K))
    if t is not None and os.environ.get("MDTF_WG_FFN_OUT") == "128" and (M, Nn, K) == (3072, 768, 8192):
        t = (128, 2, 3)                                  # (A/B switch)
    if t is not None:
        return t if (_WG_STAGES is None or t[0] != 256) else (t[0], _WG_STAGES, t[2])   # 128-row rings stay 2-deep
    kt = K // 64
    bm = 256 if M % 256 == 0 else 128
    tiles = (M // bm) * (Nn // 128)
    return bm, (3 if bm == 256 else 2), max(1, min(kt // 16, CUS // tiles))


def wg_into(gws, x, dy, dbs=None, bm=None, stages=None, splits=None, store=None):
    """gws[s] [K, Ns] fp32 += x^T @ dy[:, segment s] on the weight-gradient kernel.  x [T, K], dy [T, sum Ns]
    bf16 with unit column stride (dy may be a column slice); dbs: fp32 [Ns] slots that also receive the column
    sums of dy (the bias gradients); store[s] true: gws[s] = instead of += (the step's only write of that slot).
    Returns False when the kernel does not take the shape."""
    gws = gws if isinstance(gws, (list, tuple)) else [gws]
    T, Kin = x.shape
    Nn = dy.shape[1]
    ns = gws[0].shape[1]
    if (x.stride(1) != 1 or dy.stride(1) != 1 or Nn % 128 or Kin % 128 or T % 64 or ns * len(gws) != Nn
            or any(not g.is_contiguous() for g in gws)):
        return False
    pb, ps, psp = wg_pick(Kin, Nn, T)
    bm, stages, splits = bm or pb, stages or ps, splits or psp
    if WG_SK and splits > 1 and not N.deterministic():
        splits = -(CUS * (1 if bm == 256 else 2))      # stream-K over one (256-row) / two workgroups per CU
    if N.deterministic():
        dbs = None
    slab_n = N.fn("mdtf_gemm_wg_slab_floats_k")(Kin, Nn, T, bm, splits)
    slab = torch.empty(max(slab_n, 1), dtype=torch.float32, device=x.device) if slab_n > 0 else None
    cnt = _tickets(x.device, (Kin // bm) * (Nn // 128)) if slab_n > 0 else None
    rc = N.fn("mdtf_gemm_wg")(N.ptr(x), x.stride(0), N.ptr(dy), dy.stride(0), Kin, Nn, T, len(gws), ns,
                              ctypes.cast(_arr(gws), ctypes.c_void_p), gws[0].stride(0),
                              ctypes.cast(_arr(dbs), ctypes.c_void_p) if dbs else None, bm, stages, splits,
                              N.ptr(slab), N.ptr(cnt), sum(1 << i for i, st in enumerate(store or ()) if st),
                              N.stream_ptr())
    if rc == -2:
        return False
    N.check(min(rc, 0), "gemm_wg")
    return True
