"""The ping-pong MFMA GEMM core (``csrc/gemm_pp.hip``) as torch-facing calls.

Three layouts cover every dense-layer product without a transposed copy of anything:

* ``fwd``   ``y = act(x @ w + b)``             x [M, K], w [K, N]           (layout 0)
* ``dgrad`` ``dx (+)= dy @ w^T``               dy [M, N], w [K, N]          (layout 1)
* ``wgrad`` ``gw += x^T @ dy`` (fp32 slot)      x [M, K], dy [M, N] -> [K, N] (layout 2)

Tile codes: 0 = 256x256, 1 = 256x128, 2 = 128x256, 3 = 128x128 (rows x cols of C).  ``pick_tile``
chooses by the number of tiles the grid gets on the 256 CUs; ``TILES`` pins measured per-shape choices
(``bench/gemm_pp_probe.py``).
"""
import torch

from . import _native as N

N.register("mdtf_gemm_pp", [N.P, N.L, N.P, N.L, N.I, N.I, N.I, N.I, N.I, N.I, N.P, N.L, N.P, N.P, N.I, N.I, N.P,
                            N.L, N.P])

_TILE_DIMS = {0: (256, 256), 1: (256, 128), 2: (128, 256), 3: (128, 128)}
CUS = 256

# (layout, M, N, K) -> (tile, splits): measured choices (graph-timed on MI355X)
TILES = {}


def _waves(M, Nn, tile, splits=1):
    bm, bn = _TILE_DIMS[tile]
    t = -(-M // bm) * -(-Nn // bn) * splits
    return t, t / (CUS * -(-t // CUS))      # tiles, fraction of the last round's CUs busy ... of all rounds


def pick_tile(layout, M, Nn, K):
    """(tile, splits) for C[M][Nn] with reduction K."""
    t = TILES.get((layout, M, Nn, K))
    if t is not None:
        return t
    best = None
    for tile in (0, 1, 2, 3):
        bm, bn = _TILE_DIMS[tile]
        ntiles = -(-M // bm) * -(-Nn // bn)
        splits_opts = (1,) if layout != 2 else (1, 2, 3, 4, 6, 8)
        for sp in splits_opts:
            if K // 64 < sp * 4 and sp > 1:
                continue
            nt = ntiles * sp
            rounds = -(-nt // CUS)
            # time ~ rounds x per-tile work; smaller tiles move more LDS/L2 bytes per FLOP (x1.0 .. x1.35)
            per = (bm * bn) / float(256 * 256) * (K / sp) * {0: 1.0, 1: 1.12, 2: 1.12, 3: 1.35}[tile]
            cost = rounds * per + (0.05 * K * (sp - 1) / sp if sp > 1 else 0.0)
            if best is None or cost < best[0]:
                best = (cost, tile, sp)
    return best[1], best[2]


def _call(A, lda, B, ldb, M, Nn, K, layout, tile, splits, C=None, ldc=0, bias=None, pre=None, act=0,
          accumulate=0, Cf=None, ldcf=0):
    return N.fn("mdtf_gemm_pp")(N.ptr(A), lda, N.ptr(B), ldb, M, Nn, K, layout, tile, splits, N.ptr(C), ldc,
                                N.ptr(bias), N.ptr(pre), act, accumulate, N.ptr(Cf), ldcf, N.stream_ptr())


def fwd(x, w, bias=None, act=0, pre=None, out=None, tile=None):
    """act(x @ w + bias) in bf16 (x [M, K] row-major, w [K, N] with unit column stride)."""
    M, K = x.shape
    Nn = w.shape[1]
    y = out if out is not None else torch.empty((M, Nn), dtype=x.dtype, device=x.device)
    t = (tile, 1) if tile is not None else pick_tile(0, M, Nn, K)
    rc = _call(x, x.stride(0), w, w.stride(0), M, Nn, K, 0, t[0], 1, C=y, ldc=y.stride(0), bias=bias, pre=pre,
               act=act)
    N.check(rc, "gemm_pp fwd")
    return y


def dgrad(dy, w, out=None, accumulate=False, tile=None):
    """dy @ w^T (dy [M, N], w [K, N] row-major) -> [M, K] bf16; ``accumulate``: out += ..."""
    M, Nn = dy.shape
    K = w.shape[0]
    dx = out if out is not None else torch.empty((M, K), dtype=dy.dtype, device=dy.device)
    t = (tile, 1) if tile is not None else pick_tile(1, M, K, Nn)
    rc = _call(dy, dy.stride(0), w, w.stride(0), M, K, Nn, 1, t[0], 1, C=dx, ldc=dx.stride(0),
               accumulate=int(accumulate))
    N.check(rc, "gemm_pp dgrad")
    return dx


def wgrad_into(gw, x, dy, tile=None, splits=None):
    """gw [K, N] fp32 += x^T @ dy (x [M, K], dy [M, N] bf16, unit column strides)."""
    M, K = x.shape
    Nn = dy.shape[1]
    if tile is None:
        tile, sp = pick_tile(2, K, Nn, M)
        splits = splits or sp
    rc = _call(x, x.stride(0), dy, dy.stride(0), K, Nn, M, 2, tile, splits or 1, Cf=gw, ldcf=gw.stride(0))
    N.check(rc, "gemm_pp wgrad")
    return gw


def supported(layout, M, Nn, K):
    return K % 64 == 0 and Nn % 8 == 0 and M % 8 == 0
