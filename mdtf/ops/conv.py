"""Convolution dispatch for NHWC activations / HWIO filters on the GPU.

Per-shape backend table (``CONV_BACKEND``): the hand-written implicit-GEMM
MFMA kernels of ``csrc/conv_igemm.hip`` for the shapes where they beat the
library; MIOpen (through ``torch.nn.functional.conv2d`` on channels-last
views) otherwise.  The table is filled by ``mdtf/ops/autotune.py`` on the
target GPU; until a shape is tuned, MIOpen is used.
"""
import torch
import torch.nn.functional as F

from . import _native as N


def _miopen_conv(x, w_hwio, stride, pads, dil):
    pt, pb, pl, pr = pads
    xc = x.permute(0, 3, 1, 2)                                      # NCHW view, channels-last strides
    if not (pt == pb and pl == pr):
        xc = F.pad(xc, (pl, pr, pt, pb))
        ph, pw = 0, 0
    else:
        ph, pw = pt, pl
    wt = w_hwio.permute(3, 2, 0, 1).contiguous(memory_format=torch.channels_last)
    y = F.conv2d(xc, wt.to(x.dtype), None, stride, (ph, pw), dil)
    return y.permute(0, 2, 3, 1)


def conv2d_nhwc(x, w, stride, pads, dil, bias=None, act=None):
    y = _miopen_conv(x, w, stride, pads, dil)
    if y.stride(-1) != 1:
        y = y.contiguous()
    if bias is not None or act is not None:
        from . import kernels
        y = kernels.bias_act(y.contiguous(), bias, act)
    return y


def conv2d_dgrad_nhwc(x, w, out_shape, stride, pads):
    """conv2d_transpose = data-gradient of conv2d (filter [kh, kw, cout, cin])."""
    n, oh, ow, co = out_shape
    kh, kw, _, ci = w.shape
    pt, pb, pl, pr = pads
    xc = x.permute(0, 3, 1, 2)
    wt = w.permute(3, 2, 0, 1).to(x.dtype)                           # [cin(x), cout, kh, kw]
    y = F.conv_transpose2d(xc, wt, None, stride, 0)
    y = y[:, :, pt:pt + oh, pl:pl + ow]
    if y.shape[2] < oh or y.shape[3] < ow:
        y = F.pad(y, (0, ow - y.shape[3], 0, oh - y.shape[2]))
    return y.permute(0, 2, 3, 1).contiguous()
