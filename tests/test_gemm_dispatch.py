"""Host-side dispatch of the dense-layer kernels (no GPU): tile tables, mode switches and the CPU path of ffn()."""
import torch

from mdtf.ops import gemm as G
from mdtf.ops import nn as ops


def test_wgrad_tile_table():
    # the graph-timed per-shape 4-wave tiles (bench/dense_wgrad_sweep.py) and the small-M / default choices
    assert G._wgrad_tile(8192, 768, 3072) == (64, 128, 2, False)
    assert G._wgrad_tile(8192, 3072, 768) == (64, 128, 4, True)
    assert G._wgrad_tile(1280, 768, 768) == (64, 128, 2, False)
    assert G._wgrad_tile(8192, 768, 768) == (64, 128, 8, True)
    assert G._wgrad_tile(8192, 1024, 4096) == (64, 128, 0, True)


def test_fwd_tile_auto_keeps_library(monkeypatch):
    monkeypatch.setattr(G, "FWD_MODE", "auto")
    monkeypatch.setattr(G, "FWD_TILES", {})
    assert G._fwd_tile(8192, 768, 768, 3) is None          # auto: hipBLASLt unless the table names the shape
    monkeypatch.setattr(G, "FWD_MODE", "mdtf")
    assert G._fwd_tile(8192, 768, 768, 3) == (128, 128, 2, 2)
    assert G._fwd_tile(1000, 768, 768, 1) == (64, 128, 3, 2)
    assert G._fwd_tile(1000, 64, 64, 2) == (64, 64, 2, 2)


def test_hand_kernels_decline_cpu_tensors():
    x = torch.randn(64, 64).bfloat16()
    w = torch.randn(64, 64).bfloat16()
    assert G.hand_fwd(x, [w], None, 0) is None
    assert G.hand_dgrad_act(x, w, x, 2) is None


def test_ffn_cpu_matches_two_dense_layers():
    torch.manual_seed(0)
    x = torch.randn(8, 16, 32)
    w1, b1 = torch.randn(32, 64), torch.randn(64)
    w2, b2 = torch.randn(64, 32), torch.randn(32)
    ref = ops.dense(ops.dense(x, w1, b1, act="gelu"), w2, b2)
    assert torch.allclose(ops.ffn(x, w1, b1, w2, b2, act="gelu"), ref)
