"""Hypothesis shape sweeps of the HIP kernels against fp32 PyTorch references.

GPU only.  Each property draws random (but kernel-legal) shapes and checks the
kernel against the plain fp32 op on the same bf16-rounded inputs.  Example
counts are kept small so the whole module runs in seconds on the MI355X.
"""
import pytest
import torch

hyp = pytest.importorskip("hypothesis")
from hypothesis import HealthCheck, given, settings, strategies as st  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda"
SETTINGS = settings(max_examples=12, deadline=None, derandomize=True,
                    suppress_health_check=[HealthCheck.too_slow, HealthCheck.function_scoped_fixture])


def setup_module(module):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mdtf.ops import _native
    _native.lib()


def _rel(a, b):
    a, b = a.detach().float().cpu(), b.detach().float().cpu()
    return float((a - b).norm() / (b.norm() + 1e-12))


@SETTINGS
@given(n=st.integers(1, 4), h=st.integers(3, 17), w=st.integers(3, 17), c=st.sampled_from([64, 128, 192]),
       co=st.sampled_from([64, 128, 256, 320]), k=st.sampled_from([1, 3]), stride=st.sampled_from([1, 2]))
def test_conv_v2_matches_reference(n, h, w, c, co, k, stride):
    """v2 implicit-GEMM conv (LDS-DMA, bounds-checked zero fill) fwd/dgrad/wgrad vs fp32 conv."""
    import os
    from mdtf import nn as ops
    os.environ["MDTF_CONV"] = "mdtf2"
    try:
        torch.manual_seed(n * 1000 + h * 31 + w)
        x = torch.randn(n, h, w, c)
        wt = torch.randn(k, k, c, co) / (k * k * c) ** 0.5
        xg = x.to(DEV).bfloat16().requires_grad_(True)
        wg = wt.to(DEV).bfloat16().requires_grad_(True)
        y = ops.conv2d(xg, wg, stride, "SAME")
        xc = x.bfloat16().float().requires_grad_(True)
        wc = wt.bfloat16().float().requires_grad_(True)
        yr = ops.conv2d(xc, wc, stride, "SAME")
        assert _rel(y, yr) < 1e-2
        dy = torch.randn(yr.shape)
        y.backward(dy.to(DEV).bfloat16())
        yr.backward(dy.bfloat16().float())
        assert _rel(xg.grad, xc.grad) < 2e-2
        assert _rel(wg.grad, wc.grad) < 2e-2
    finally:
        os.environ.pop("MDTF_CONV", None)


@SETTINGS
@given(rows=st.integers(1, 300), h=st.sampled_from([64, 128, 256, 512, 768, 1024]), res=st.booleans(),
       p=st.sampled_from([0.0, 0.1]))
def test_layernorm_matches_reference(rows, h, res, p):
    from mdtf.ops import transformer as T
    torch.manual_seed(rows + h)
    x = torch.randn(rows, h)
    r = torch.randn(rows, h) if res else None
    g = torch.rand(h) + 0.5
    b = torch.randn(h)
    xg = x.to(DEV).bfloat16()
    rg = r.to(DEV).bfloat16() if res else None
    y = T._LayerNorm.apply(xg, rg, g.to(DEV), b.to(DEV), 1e-12, p, 12345)
    if p:
        from test_kernels_gpu import _hash_keep
        keep = _hash_keep(12345, rows * h, p).view(rows, h).float()
        xs = x.bfloat16().float() * keep / (1 - p)
    else:
        xs = x.bfloat16().float()
    s = xs + (r.bfloat16().float() if res else 0)
    yr = torch.nn.functional.layer_norm(s, (h,), g, b, 1e-12)
    assert _rel(y, yr) < 2e-2


@SETTINGS
@given(m=st.integers(1, 5000), c=st.sampled_from([8, 64, 72, 768, 3072, 10, 30]))
def test_colsum_matches_reference(m, c):
    from mdtf.ops import kernels as K
    x = torch.randn(m, c)
    out = torch.zeros(c, device=DEV)
    K.colsum_into(x.to(DEV).bfloat16(), out)
    assert _rel(out, x.bfloat16().float().sum(0)) < 1e-4


@SETTINGS
@given(b=st.integers(1, 3), heads=st.integers(1, 4), p=st.sampled_from([0.0, 0.1]))
def test_fused_attention_matches_reference(b, heads, p):
    from mdtf.ops import transformer as T
    from test_kernels_gpu import _attn_keep_mask
    S, dh = 128, 64
    H = heads * dh
    torch.manual_seed(b * 7 + heads)
    qkv = torch.randn(b * S, 3 * H) * 0.5
    mask = (torch.rand(b, S) < 0.2).float() * -10000.0
    out = T._FusedAttention.apply(qkv.to(DEV).bfloat16(), mask.to(DEV), b, S, heads, p, 777)
    q, k, v = qkv.bfloat16().float().reshape(b, S, 3, heads, dh).unbind(2)
    q, k, v = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
    pr = torch.softmax(q @ k.transpose(-1, -2) / dh ** 0.5 + mask[:, None, None, :], -1)
    if p:
        pr = pr * _attn_keep_mask(777, b, heads, S, p) / (1 - p)
    ref = (pr @ v).transpose(1, 2).reshape(b * S, H)
    assert _rel(out, ref) < 1.5e-2


@SETTINGS
@given(m=st.integers(1, 700), c=st.sampled_from([8, 64, 200, 768]), act=st.sampled_from(["relu", "gelu", None]))
def test_dense_bias_act_matches_reference(m, c, act):
    from mdtf import nn as ops
    torch.manual_seed(m + c)
    x = torch.randn(m, 96)
    w = torch.randn(96, c) / 10
    b = torch.randn(c).bfloat16().float()
    y = ops.dense(x.to(DEV).bfloat16(), w.to(DEV).bfloat16(), b.to(DEV), act=act)
    yr = x.bfloat16().float() @ w.bfloat16().float() + b
    if act == "relu":
        yr = torch.relu(yr)
    elif act == "gelu":
        yr = torch.nn.functional.gelu(yr, approximate="tanh")
    assert _rel(y, yr) < 1.5e-2
