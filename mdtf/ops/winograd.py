"""Non-fused Winograd F(2x2, 3x3) convolution (``csrc/winograd.hip`` transforms + hand-written MFMA GEMMs).

The reference exposes Winograd only as an environment toggle for cuDNN
(``TF_ENABLE_WINOGRAD_NONFUSED=1`` in ``distribute.py``).  Here
the same switch (or ``MDTF_WINOGRAD=1`` / ``MDTF_CONV=winograd``) routes every
eligible 3x3 stride-1 forward and data-gradient pass through this algorithm:
input transform -> 16 GEMMs -> output transform, each transform one HIP kernel.
The 16 GEMMs [T tiles x C] x [C x K] run on the weight-stationary MFMA kernel
(``csrc/conv_ws.hip`` as a 1x1 convolution over the T tiles; the transformed
filters transposed once to [16][K][C]); shapes it does not take (C % 32,
K % 64) use a batched hipBLASLt GEMM.  Weight gradients stay on the implicit-GEMM kernel.  The autotuner
(``bench/conv_autotune.py``) measures it per shape next to the other backends;
on MI355X the implicit GEMM usually wins because the transformed tensors cost
more HBM traffic than the 2.25x MFMA saving (profiles/conv_autotune_*.md).
"""
import os

import torch

from . import _native as N

N.register("mdtf_wino_input", [N.P, N.P] + [N.I] * 8 + [N.P])
N.register("mdtf_wino_filter", [N.P, N.P, N.I, N.I, N.I, N.P])
N.register("mdtf_wino_output", [N.P, N.P, N.I, N.I, N.I, N.I, N.P])


def enabled():
    for var in ("TF_ENABLE_WINOGRAD_NONFUSED", "MDTF_WINOGRAD"):
        if os.environ.get(var, "0").lower() in ("1", "true", "yes", "on"):
            return True
    return os.environ.get("MDTF_CONV", "") == "winograd"


def eligible(w_shape, stride, pads, dil, c, co):
    kh, kw = w_shape[0], w_shape[1]
    return (kh == 3 and kw == 3 and tuple(stride) == (1, 1) and tuple(dil) == (1, 1)
            and all(0 <= p <= 2 for p in pads) and c % 8 == 0 and co % 8 == 0)


def _conv(x, w, out_hw, ph, pw, flip):
    n, h, wd, c = x.shape
    k = w.shape[2] if flip else w.shape[3]
    oh, ow = out_hw
    th, tw = (oh + 1) // 2, (ow + 1) // 2
    t = n * th * tw
    v = torch.empty((16, t, c), dtype=x.dtype, device=x.device)
    N.check(N.fn("mdtf_wino_input")(N.ptr(x), N.ptr(v), n, h, wd, c, oh, ow, ph, pw, N.stream_ptr()), "wino_input")
    u = torch.empty((16, c, k), dtype=x.dtype, device=x.device)
    N.check(N.fn("mdtf_wino_filter")(N.ptr(w), N.ptr(u), w.shape[2], w.shape[3], int(flip), N.stream_ptr()),
            "wino_filter")
    m = _gemm16(v, u)                         # [16, T, K], fp32 accumulation
    y = torch.empty((n, oh, ow, k), dtype=x.dtype, device=x.device)
    N.check(N.fn("mdtf_wino_output")(N.ptr(m), N.ptr(y), n, oh, ow, k, N.stream_ptr()), "wino_output")
    return y


WS_TILE = (2, 8, 1, 4)


def _gemm16(v, u):
    """m[b] = v[b] @ u[b] for the 16 transform positions: hand-written kernel where it applies."""
    from . import conv as C
    from . import kernels
    b, t, c = v.shape
    k = u.shape[2]
    if (N.use_native(v) and v.dtype == torch.bfloat16 and C.ws_ok("fwd", c, k, (1, 1), 1, 1)
            and C.ws_depth_ok(c, WS_TILE[3])):
        ut = kernels.transpose_brs(u, b, c, k)          # [16][K][C]: the kernel's A operand layout
        m = torch.empty((b, t, k), dtype=v.dtype, device=v.device)
        for i in range(b):
            C.ws_fwd(v[i].view(1, 1, t, c), ut[i], 1, 1, (1, t), (1, 1), (0, 0, 0, 0), (1, 1), WS_TILE,
                     out=m[i].view(1, 1, t, k))
        return m
    return torch.bmm(v, u)                  # hipBLASLt


def winograd_fwd(x, w, out_hw, pads):
    """NHWC x, HWIO 3x3 w, pads (top, bottom, left, right) -> y [N, OH, OW, Co]."""
    return _conv(x.contiguous(), w.contiguous(), out_hw, pads[0], pads[2], False)


def winograd_dgrad(dy, w, x_shape, pads):
    """DX of a stride-1 3x3 conv: correlation of DY (padded 2 - pad) with the rotated, transposed filter."""
    return _conv(dy.contiguous(), w.contiguous(), (x_shape[1], x_shape[2]), 2 - pads[0], 2 - pads[2], True)


def reference(x, w, pads):
    """The same algorithm in plain fp32 torch (CPU-testable): F(2x2, 3x3) tiles of ``x`` NHWC, ``w`` HWIO."""
    bt = torch.tensor([[1, 0, -1, 0], [0, 1, 1, 0], [0, -1, 1, 0], [0, 1, 0, -1]], dtype=torch.float32)
    g = torch.tensor([[1, 0, 0], [.5, .5, .5], [.5, -.5, .5], [0, 0, 1]], dtype=torch.float32)
    at = torch.tensor([[1, 1, 1, 0], [0, 1, -1, -1]], dtype=torch.float32)
    n, h, wd, c = x.shape
    oh, ow = h + pads[0] + pads[1] - 2, wd + pads[2] + pads[3] - 2
    th, tw = (oh + 1) // 2, (ow + 1) // 2
    # pad to (2 th + 2) x (2 tw + 2): the conv padding plus the odd-size tile tail
    xp = torch.nn.functional.pad(x.float(), (0, 0, pads[2], pads[3] + 2 * tw - ow, pads[0], pads[1] + 2 * th - oh))
    d = xp.unfold(1, 4, 2).unfold(2, 4, 2)                    # [n, th, tw, c, 4, 4]
    v = torch.einsum("ij,ntwcjk,lk->ntwcil", bt, d, bt)       # B^T d B
    u = torch.einsum("ij,jkco,lk->coil", g, w.float(), g)     # G g G^T   [c, o, 4, 4]
    m = torch.einsum("ntwcil,coil->ntwoil", v, u)
    y = torch.einsum("ij,ntwojk,lk->ntwoil", at, m, at)       # [n, th, tw, o, 2, 2]
    y = y.permute(0, 1, 4, 2, 5, 3).reshape(n, 2 * th, 2 * tw, -1)
    return y[:, :oh, :ow]
