"""CPU-side checks of the ping-pong GEMM core's host logic (mdtf/ops/mm.py) and of the fused multi-update
optimizer path the async parameter server uses (mdtf/ops/optim.py apply_multi_)."""
import torch

from mdtf.ops import mm
from mdtf.ops import optim


def test_pick_tile_fills_the_cus_on_bert_shapes():
    # BERT-base at batch 64 x 128: every forward / data-gradient shape gets a tile whose grid is whole waves of the
    # 256 CUs (or the cheapest modelled choice), and the transposed operands' extents are tile multiples
    for (layout, M, N, K) in [(0, 8192, 2304, 768), (0, 8192, 768, 768), (0, 8192, 3072, 768), (0, 8192, 768, 3072),
                              (1, 8192, 768, 2304), (1, 8192, 768, 3072), (1, 8192, 3072, 768)]:
        tile, sp = mm.pick_tile(layout, M, N, K)
        bm, bn = mm._TILE_DIMS[tile]
        assert sp == 1
        assert mm._valid(layout, tile, M, N)
        tiles = -(-M // bm) * -(-N // bn)
        assert tiles >= 128, (layout, M, N, K, tile)


def test_pick_tile_respects_transposed_operand_extents():
    # wgrad: C rows (= K features) and columns must be tile multiples
    tile, sp = mm.pick_tile(2, 768, 2304, 8192)
    bm, bn = mm._TILE_DIMS[tile]
    assert 768 % bm == 0 and 2304 % bn == 0 and sp >= 1
    assert mm.pick_tile(2, 320, 100, 64) is None          # nothing tiles 320 x 100
    # segmented forward: a tile never straddles two segments
    tile, _ = mm.pick_tile(0, 8192, 2304, 768, seg_cols=768)
    assert 768 % mm._TILE_DIMS[tile][1] == 0


def _sequential(kind, master, grads, s1, s2, lrs, lr_ts, **kw):
    for g, lr, lt in zip(grads, lrs, lr_ts):
        if kind == "momentum":
            optim.momentum_(master, g.float(), s1, None, lr, kw["momentum"], 1.0, kw.get("weight_decay", 0.0))
        elif kind == "adam":
            gg = g.float()
            s1.mul_(kw["beta1"]).add_(gg, alpha=1 - kw["beta1"])
            s2.mul_(kw["beta2"]).addcmul_(gg, gg, value=1 - kw["beta2"])
            master.sub_(lt * s1 / (s2.sqrt() + kw["epsilon"]))
        else:
            optim.sgd_(master, g.float(), None, lr)


def test_apply_multi_equals_sequential_updates():
    torch.manual_seed(0)
    for kind in ("sgd", "momentum", "adam"):
        w0 = torch.randn(256)
        grads = [torch.randn(256).to(torch.bfloat16) for _ in range(3)]
        lrs, lrts = [0.1, 0.05, 0.02], [0.01, 0.009, 0.008]
        kw = dict(momentum=0.9, beta1=0.9, beta2=0.999, epsilon=1e-8)
        a, b = w0.clone(), w0.clone()
        sa1, sa2, sb1, sb2 = (torch.zeros(256) for _ in range(4))
        optim.apply_multi_(kind, a, grads, sa1, sa2, None, lrs, lrts, **kw)
        _sequential(kind, b, grads, sb1, sb2, lrs, lrts, **kw)
        assert torch.allclose(a, b, atol=1e-6), kind


def test_wg_pick_table_and_fallback_fill_the_cus():
    # measured table entries come back as stored (256-row tiles: 3-stage ring; 128-row: 2-stage)
    for key, val in mm.WG_TILES.items():
        if mm._WG_STAGES is None:
            assert mm.wg_pick(*key) == val
    # fallback: 256-row tiles when the rows allow it, split so tiles x splits <= 256 CUs, >= 16 K-tiles per split
    for (M, Nn, K) in [(512, 1024, 8192), (640, 384, 4096), (2048, 2048, 4096), (128, 128, 64 * 8)]:
        bm, st, sp = mm.wg_pick(M, Nn, K)
        assert bm == (256 if M % 256 == 0 else 128) and st == (3 if bm == 256 else 2)
        tiles = (M // bm) * (Nn // 128)
        assert sp >= 1 and (sp == 1 or (tiles * sp <= mm.CUS and (K // 64) // sp >= 16)), (M, Nn, K, sp)


def test_wg_route_shape_gate():
    from mdtf.ops import gemm
    x = torch.empty(8192, 768, dtype=torch.bfloat16)
    assert gemm._wg_ok(x, torch.empty(8192, 2304, dtype=torch.bfloat16))       # q|k|v
    assert gemm._wg_ok(torch.empty(8192, 3072, dtype=torch.bfloat16), torch.empty(8192, 768, dtype=torch.bfloat16))
    assert not gemm._wg_ok(x, torch.empty(8192, 100, dtype=torch.bfloat16))    # N not a 128-multiple
    assert not gemm._wg_ok(x[:2048], torch.empty(2048, 2304, dtype=torch.bfloat16))   # too few tokens
    assert not gemm._wg_ok(torch.empty(8032, 768, dtype=torch.bfloat16), torch.empty(8032, 2304, dtype=torch.bfloat16))
