"""Winograd F(2x2, 3x3) convolution (the reference's TF_ENABLE_WINOGRAD_NONFUSED toggle).

CPU: the transform algebra (``mdtf.ops.winograd.reference``) against torch's conv2d.
GPU: the HIP transforms + batched GEMM, forward and data gradient, and the toggle routing a
training step's 3x3 stride-1 convolutions through it.
"""
import pytest
import torch

from mdtf.ops import winograd as Wg


def _conv_ref(x, w, pads):
    xn = torch.nn.functional.pad(x.permute(0, 3, 1, 2).float(), (pads[2], pads[3], pads[0], pads[1]))
    return torch.nn.functional.conv2d(xn, w.float().permute(3, 2, 0, 1)).permute(0, 2, 3, 1)


@pytest.mark.parametrize("shape,pads", [((2, 9, 9, 8, 16), (1, 1, 1, 1)), ((1, 8, 7, 8, 8), (0, 0, 0, 0)),
                                        ((2, 6, 11, 16, 8), (1, 1, 1, 1)), ((1, 7, 6, 8, 8), (0, 1, 0, 1))])
def test_winograd_reference_algebra(shape, pads):
    n, h, w, c, k = shape
    torch.manual_seed(h * 10 + w)
    x = torch.randn(n, h, w, c)
    wt = torch.randn(3, 3, c, k)
    y = Wg.reference(x, wt, pads)
    assert (y - _conv_ref(x, wt, pads)).abs().max() < 1e-4


def test_winograd_toggle_and_eligibility(monkeypatch):
    monkeypatch.delenv("MDTF_WINOGRAD", raising=False)
    monkeypatch.delenv("TF_ENABLE_WINOGRAD_NONFUSED", raising=False)
    assert not Wg.enabled()
    monkeypatch.setenv("TF_ENABLE_WINOGRAD_NONFUSED", "1")
    assert Wg.enabled()
    assert Wg.eligible((3, 3), (1, 1), (1, 1, 1, 1), (1, 1), 64, 64)
    assert not Wg.eligible((3, 3), (2, 2), (1, 1, 1, 1), (1, 1), 64, 64)
    assert not Wg.eligible((1, 1), (1, 1), (0, 0, 0, 0), (1, 1), 64, 64)
    assert not Wg.eligible((3, 3), (1, 1), (1, 1, 1, 1), (1, 1), 3, 64)
    from mdtf.ops import conv as C
    assert C.choose("fwd", (2, 8, 8, 64), (3, 3, 64, 64), (1, 1), (1, 1, 1, 1), (1, 1)) == ("winograd",)
    assert C.choose("wgrad", (2, 8, 8, 64), (3, 3, 64, 64), (1, 1), (1, 1, 1, 1), (1, 1))[0] != "winograd"


def _rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


@pytest.mark.gpu
@pytest.mark.parametrize("shape,pads", [((2, 14, 14, 64, 128), (1, 1, 1, 1)), ((3, 9, 7, 72, 64), (1, 1, 1, 1)),
                                        ((2, 8, 8, 64, 64), (0, 0, 0, 0)), ((1, 7, 7, 128, 256), (0, 1, 0, 1))])
def test_winograd_hip_fwd_dgrad(shape, pads):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    n, h, w, c, k = shape
    torch.manual_seed(c + k)
    x = torch.randn(n, h, w, c).bfloat16()
    wt = (torch.randn(3, 3, c, k) / (9 * c) ** 0.5).bfloat16()
    oh, ow = h + pads[0] + pads[1] - 2, w + pads[2] + pads[3] - 2
    y = Wg.winograd_fwd(x.cuda(), wt.cuda(), (oh, ow), pads)
    assert _rel(y, _conv_ref(x, wt, pads)) < 1.5e-2
    dy = torch.randn(n, oh, ow, k).bfloat16()
    xr = x.float().requires_grad_(True)
    _conv_ref(xr, wt, pads).backward(dy.float())
    dx = Wg.winograd_dgrad(dy.cuda(), wt.cuda(), x.shape, pads)
    assert _rel(dx, xr.grad) < 1.5e-2


@pytest.mark.gpu
def test_winograd_toggle_training_step(monkeypatch):
    """conv2d under the toggle: forward and both gradients vs the fp32 reference."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mdtf import nn as ops
    monkeypatch.setenv("TF_ENABLE_WINOGRAD_NONFUSED", "1")
    torch.manual_seed(1)
    x = torch.randn(4, 12, 12, 64)
    w = torch.randn(3, 3, 64, 128) / 24.0
    xg = x.cuda().bfloat16().requires_grad_(True)
    wg = w.cuda().bfloat16().requires_grad_(True)
    y = ops.conv2d(xg, wg, 1, "SAME")
    xc = x.bfloat16().float().requires_grad_(True)
    wc = w.bfloat16().float().requires_grad_(True)
    yr = ops.conv2d(xc, wc, 1, "SAME")
    assert _rel(y, yr) < 1.5e-2
    dy = torch.randn(yr.shape)
    y.backward(dy.cuda().bfloat16())
    yr.backward(dy.bfloat16().float())
    assert _rel(xg.grad, xc.grad) < 2e-2
    assert _rel(wg.grad, wc.grad) < 2e-2
