"""Numerics of every HIP kernel vs a plain PyTorch fp32 reference (GPU only)."""
import pytest
import torch

from mdtf.ops import _native
from mdtf.ops import nn as ops

pytestmark = pytest.mark.gpu

DEV = "cuda"


def setup_module(module):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _native.lib()  # must load: no silent fallback


def _rel(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _ref_bn(x, gamma, beta, res, relu, eps):
    xf = x.float()
    C = xf.shape[-1]
    x2 = xf.reshape(-1, C)
    mean = x2.mean(0)
    var = x2.var(0, unbiased=False)
    y = (x2 - mean) * torch.rsqrt(var + eps) * gamma + beta
    y = y.reshape(xf.shape)
    if res is not None:
        y = y + res.float()
    return torch.relu(y) if relu else y


@pytest.mark.parametrize("shape,relu,with_res", [((8, 14, 14, 64), True, False), ((4, 7, 7, 256), True, True),
                                                  ((16, 3, 3, 2048), False, True), ((2, 28, 28, 128), False, False)])
def test_batch_norm_fwd_bwd(shape, relu, with_res):
    torch.manual_seed(0)
    C = shape[-1]
    x = (torch.randn(shape) * 2 + 0.5).to(DEV).bfloat16().requires_grad_(True)
    res = torch.randn(shape).to(DEV).bfloat16().requires_grad_(True) if with_res else None
    gamma = (torch.rand(C) + 0.5).to(DEV).requires_grad_(True)
    beta = torch.randn(C).to(DEV).requires_grad_(True)
    mm = torch.zeros(C, device=DEV)
    mv = torch.ones(C, device=DEV)
    y = ops.batch_norm(x, gamma, beta, mm, mv, True, 0.9, 1e-5, relu, res)
    xr = x.detach().float().cpu().requires_grad_(True)
    rr = res.detach().float().cpu().requires_grad_(True) if with_res else None
    gr = gamma.detach().cpu().requires_grad_(True)
    br = beta.detach().cpu().requires_grad_(True)
    yr = _ref_bn(xr, gr, br, rr, relu, 1e-5)
    assert _rel(y, yr) < 1e-2
    dy = torch.randn(shape)
    y.backward(dy.to(DEV).bfloat16())
    yr.backward(dy.bfloat16().float())
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(gamma.grad, gr.grad) < 2e-2
    assert _rel(beta.grad, br.grad) < 2e-2
    if with_res:
        assert _rel(res.grad, rr.grad) < 2e-2
    m = xr.detach().reshape(-1, C).mean(0)
    assert _rel(mm, 0.1 * m) < 1e-2
    # eval path uses the moving statistics
    ye = ops.batch_norm(x.detach(), gamma.detach(), beta.detach(), mm, mv, False, 0.9, 1e-5, relu, None)
    xf = x.detach().float().cpu()
    ref = (xf - mm.cpu()) * torch.rsqrt(mv.cpu() + 1e-5) * gamma.detach().cpu() + beta.detach().cpu()
    assert _rel(ye, torch.relu(ref) if relu else ref) < 1e-2


@pytest.mark.parametrize("shape", [(8, 14, 14, 256), (16, 2, 2, 2048), (4, 28, 28, 512)])
def test_batch_norm_dual_deferred_shortcut(shape):
    """relu(BN(x) + BN2(r)) in one apply pass (the projection shortcut's BN deferred into the residual BN,
    ops.bn._BNTrainDual) vs fp32 autograd: output, dx, dr, all four BN parameter gradients and both
    moving means."""
    from mdtf.ops import bn as B
    torch.manual_seed(3)
    C = shape[-1]
    x = (torch.randn(shape) * 2 + 0.5).to(DEV).bfloat16().requires_grad_(True)
    r = (torch.randn(shape) * 0.7 - 0.2).to(DEV).bfloat16().requires_grad_(True)
    ps = [(torch.rand(C) + 0.5).to(DEV).requires_grad_(True), torch.randn(C).to(DEV).requires_grad_(True),
          (torch.rand(C) + 0.5).to(DEV).requires_grad_(True), torch.randn(C).to(DEV).requires_grad_(True)]
    mm, mv, mm2, mv2 = torch.zeros(C, device=DEV), torch.ones(C, device=DEV), torch.zeros(C, device=DEV), \
        torch.ones(C, device=DEV)

    def partials(t):     # [2][1][C] fp32 partial sums, as a conv epilogue would emit them (one slot)
        t2 = t.detach().float().reshape(-1, C)
        return (t2.sum(0, keepdim=True).contiguous(), (t2 * t2).sum(0, keepdim=True).contiguous(), 1)
    y = B._BNTrainDual.apply(x, ps[0], ps[1], mm, mv, r, ps[2], ps[3], mm2, mv2, 0.9, 1e-5, partials(x), partials(r))
    xr = x.detach().float().cpu().requires_grad_(True)
    rr = r.detach().float().cpu().requires_grad_(True)
    pr = [p.detach().cpu().requires_grad_(True) for p in ps]
    yr = torch.relu(_ref_bn(xr, pr[0], pr[1], None, False, 1e-5) + _ref_bn(rr, pr[2], pr[3], None, False, 1e-5))
    assert _rel(y, yr) < 1e-2
    dy = torch.randn(shape)
    y.backward(dy.to(DEV).bfloat16())
    yr.backward(dy.bfloat16().float())
    assert _rel(x.grad, xr.grad) < 2e-2
    assert _rel(r.grad, rr.grad) < 2e-2
    for p, q in zip(ps, pr):
        assert _rel(p.grad, q.grad) < 2e-2
    assert _rel(mm, 0.1 * xr.detach().reshape(-1, C).mean(0)) < 1e-2
    assert _rel(mm2, 0.1 * rr.detach().reshape(-1, C).mean(0)) < 1e-2


@pytest.mark.parametrize("is_max", [True, False])
@pytest.mark.parametrize("k,s,pad", [(3, 2, "SAME"), (2, 2, "SAME"), (3, 1, "VALID")])
def test_pool(is_max, k, s, pad):
    torch.manual_seed(1)
    x = torch.randn(4, 15, 15, 64)
    xg = x.to(DEV).bfloat16().requires_grad_(True)
    xc = x.bfloat16().float().requires_grad_(True)
    f = ops.max_pool if is_max else ops.avg_pool
    y = f(xg, k, s, pad)
    yr = f(xc, k, s, pad)
    assert y.shape == yr.shape
    assert _rel(y, yr) < 1e-2
    dy = torch.randn(yr.shape)
    y.backward(dy.to(DEV).bfloat16())
    yr.backward(dy.bfloat16().float())
    assert _rel(xg.grad, xc.grad) < 2e-2


def test_global_avg_pool():
    x = torch.randn(8, 7, 7, 512)
    xg = x.to(DEV).bfloat16().requires_grad_(True)
    xc = x.bfloat16().float().requires_grad_(True)
    y = ops.global_avg_pool(xg)
    yr = xc.mean(dim=(1, 2))
    assert _rel(y, yr) < 1e-2
    dy = torch.randn(8, 512)
    y.backward(dy.to(DEV).bfloat16())
    yr.backward(dy.bfloat16().float())
    assert _rel(xg.grad, xc.grad) < 1e-2


@pytest.mark.parametrize("dtype,N,K", [(torch.bfloat16, 37, 1000), (torch.float32, 37, 1000),
                                       (torch.bfloat16, 300, 30522), (torch.bfloat16, 5, 4096)])
def test_softmax_xent(dtype, N, K):
    """K >= 2048 bf16 rows take the one-block-per-row online-softmax kernel."""
    torch.manual_seed(2)
    logits = torch.randn(N, K) * 3
    labels = torch.randint(0, K, (N,))
    lg = logits.to(DEV).to(dtype).requires_grad_(True)
    lc = logits.to(dtype).float().requires_grad_(True)
    l = ops.sparse_softmax_cross_entropy_with_logits(labels.to(DEV), lg)
    lr = torch.nn.functional.cross_entropy(lc, labels, reduction="none")
    assert _rel(l, lr) < 1e-3
    l.mean().backward()
    lr.mean().backward()
    assert _rel(lg.grad, lc.grad) < 2e-2


def test_softmax_xent_strided_rows():
    """Logits as a [rows, 30522] view of [rows, 30720] rows (the padded MLM decoder): the 16-B vector forward and
    backward kernels, the gradient handed back as the same view of a zero-padded buffer."""
    from mdtf.ops import gemm
    torch.manual_seed(3)
    N, K, LD = 67, 30522, 30720
    full = (torch.randn(N, LD) * 3).bfloat16()
    labels = torch.randint(0, K, (N,))
    lp = full.to(DEV).requires_grad_(True)
    lg = lp[:, :K]
    l = ops.sparse_softmax_cross_entropy_with_logits(labels.to(DEV), lg)
    lc = full[:, :K].float().requires_grad_(True)
    lr = torch.nn.functional.cross_entropy(lc, labels, reduction="none")
    assert _rel(l, lr) < 1e-3
    l.mean().backward()
    lr.mean().backward()
    assert _rel(lp.grad[:, :K], lc.grad) < 2e-2
    assert not lp.grad[:, K:].any()
    gemm._PADDED_GRADS.clear()


def test_softmax_xent_unaligned_strided_rows_zero_pad():
    """a strided logits view that is NOT 16-B aligned runs the generic backward kernel, which does not
    touch the pad columns; the gradient buffer registered as zero-padded must still be zero there (the tied decoder
    reads whole rows, 0 * NaN would poison dh)."""
    import types
    from mdtf.ops import gemm, kernels
    torch.manual_seed(4)
    N, K, LD = 9, 3000, 3008
    full = (torch.randn(N, LD + 1) * 3).bfloat16().to(DEV)
    lg = full.as_strided((N, K), (LD, 1), storage_offset=1)        # 2-B offset: the vector path is refused
    assert lg.data_ptr() % 16 and lg.stride(0) == LD
    labels = torch.randint(0, K, (N,), device=DEV)
    loss = kernels.softmax_xent(lg, labels)
    lse = torch.logsumexp(lg.float(), 1)
    ctx = types.SimpleNamespace(saved_tensors=(lg, labels, lse))
    for _ in range(3):                   # the caching allocator hands back dirty blocks: poison one first
        torch.full((N, LD), float("nan"), dtype=torch.bfloat16, device=DEV)
    g, _ = kernels._Xent.backward(ctx, torch.ones(N, device=DEV))
    whole = g.as_strided((N, LD), (LD, 1))
    assert not whole[:, K:].isnan().any() and not whole[:, K:].any()
    ref = torch.softmax(lg.float(), 1)
    ref[torch.arange(N, device=DEV), labels] -= 1
    assert _rel(g, ref) < 2e-2
    assert torch.isfinite(loss).all()
    gemm._PADDED_GRADS.clear()


@pytest.mark.parametrize("act", ["relu", "gelu", None])
@pytest.mark.parametrize("C", [64, 10])
def test_bias_act(act, C):
    torch.manual_seed(5)
    x = torch.randn(33, C)
    b = torch.randn(C).bfloat16().float()     # the GEMM epilogue adds the bf16 bias
    xg = x.to(DEV).bfloat16().requires_grad_(True)
    bg = b.to(DEV).requires_grad_(True)
    y = ops.dense(xg, torch.eye(C, device=DEV), bg, act=act)
    xc = x.bfloat16().float().requires_grad_(True)
    bc = b.clone().requires_grad_(True)
    yr = xc + bc
    if act == "relu":
        yr = torch.relu(yr)
    elif act == "gelu":
        yr = torch.nn.functional.gelu(yr, approximate="tanh")
    assert _rel(y, yr) < 1e-2
    dy = torch.randn(33, C)
    y.backward(dy.to(DEV).bfloat16())
    yr.backward(dy.bfloat16().float())
    assert _rel(xg.grad, xc.grad) < 2e-2
    assert _rel(bg.grad, bc.grad) < 2e-2


def test_layout_transform():
    from mdtf.ops import kernels
    x = torch.randn(3, 17, 9, 11)
    for dt in (torch.float32, torch.bfloat16):
        xg = x.to(DEV).to(dt)
        y = kernels.nchw_to_nhwc(xg)
        assert torch.equal(y.cpu(), x.to(dt).permute(0, 2, 3, 1))
        assert torch.equal(kernels.nhwc_to_nchw(y).cpu(), x.to(dt))


def test_lrn():
    x = torch.randn(2, 5, 5, 32)
    xg = x.to(DEV).bfloat16().requires_grad_(True)
    xc = x.bfloat16().float().requires_grad_(True)
    y = ops.lrn(xg, 4, 1.0, 0.001 / 9, 0.75)
    yr = ops.lrn(xc, 4, 1.0, 0.001 / 9, 0.75)
    assert _rel(y, yr) < 1e-2
    dy = torch.randn(x.shape)
    y.backward(dy.to(DEV).bfloat16())
    yr.backward(dy.bfloat16().float())
    assert _rel(xg.grad, xc.grad) < 2e-2


@pytest.mark.parametrize("kind", ["sgd", "momentum", "adam"])
def test_fused_optimizers(kind):
    from mdtf.ops import optim
    torch.manual_seed(3)
    n = 4096
    w = torch.randn(n)
    g = torch.randn(n)
    s1 = torch.randn(n).abs()
    s2 = torch.randn(n).abs()
    wg, gg, s1g, s2g = w.to(DEV), g.to(DEV), s1.to(DEV), s2.to(DEV)
    shadow = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    if kind == "sgd":
        optim.sgd_(wg, gg, shadow, 0.1, 0.5, 1e-2)
        optim.sgd_(w, g, None, 0.1, 0.5, 1e-2)
    elif kind == "momentum":
        optim.momentum_(wg, gg, s1g, shadow, 0.1, 0.9, 0.5, 1e-2, False)
        optim.momentum_(w, g, s1, None, 0.1, 0.9, 0.5, 1e-2, False)
    else:
        optim.adam_(wg, gg, s1g, s2g, shadow, 1e-3, 0.9, 0.999, 1e-8, 3, 0.5, 1e-2, True)
        optim.adam_(w, g, s1, s2, None, 1e-3, 0.9, 0.999, 1e-8, 3, 0.5, 1e-2, True)
    assert _rel(wg, w) < 1e-6
    assert _rel(shadow, w) < 1e-2


def test_conv2d_matches_reference():
    torch.manual_seed(4)
    x = torch.randn(2, 9, 9, 16)
    w = torch.randn(3, 3, 16, 32) * 0.1
    for stride, pad in ((1, "SAME"), (2, (1, 1)), (2, "SAME"), (1, "VALID")):
        y = ops.conv2d(x.to(DEV).bfloat16(), w.to(DEV).bfloat16(), stride, pad)
        yr = ops.conv2d(x.bfloat16().float(), w.bfloat16().float(), stride, pad)
        assert y.shape == yr.shape
        assert _rel(y, yr) < 1e-2


def test_resnet_train_step_gpu():
    """A tiny ResNet step through the whole engine on the GPU kernels."""
    import mdtf
    from mdtf.data.loaders import SyntheticDataLoader
    from mdtf.models import ResNet, SoftmaxCrossEntropyLoss
    from mdtf.runtime import Net, Tower
    from mdtf.train import variables as V
    store = V.get_store()
    store.device = torch.device(DEV)
    store.compute_dtype = torch.bfloat16
    loader = SyntheticDataLoader(shape=(64, 64, 3), num_classes=10, dtype=torch.bfloat16)
    loader.batch_size = 8
    raw, gt = loader.load_train_batch()
    opt = mdtf.train.MomentumOptimizer(0.05, 0.9)
    gs = mdtf.train.get_or_create_global_step()
    tg = []
    tower = Tower(Net(ResNet(50, num_classes=10)), "tower_0/", tg, raw, gt, SoftmaxCrossEntropyLoss(), opt,
                  batch_size=8)
    _, loss, _ = tower.process()
    train_op = opt.apply_gradients(Tower.average_gradients(tg), global_step=gs)
    sess = mdtf.train.MonitoredTrainingSession(log_step_count_steps=0)
    losses = []
    for _ in range(8):
        sess.run(train_op)
        losses.append(float(sess.run(loss)))
    assert all(l == l for l in losses)
    assert losses[-1] < losses[0]


CONV_CASES = [
    # (N, H, W, C, KH, KW, CO, stride, padding)
    (2, 9, 9, 16, 3, 3, 32, 1, "SAME"),
    (3, 14, 14, 64, 1, 1, 256, 1, "VALID"),
    (2, 15, 15, 32, 3, 3, 64, 2, (1, 1)),
    (2, 16, 16, 64, 1, 1, 128, 2, "VALID"),
    (1, 13, 11, 8, 3, 3, 72, 1, "SAME"),           # K=72 (not a multiple of 32), Cout=72
    (2, 20, 20, 8, 7, 7, 64, 2, (3, 3)),           # stem-like 7x7/2 with 8 channels
    (5, 7, 7, 128, 3, 3, 128, 1, "SAME"),          # M tail (245 rows)
    (2, 14, 14, 64, 3, 3, 128, 2, (1, 1)),         # v2: strided 3x3 (dgrad divisibility path)
    (3, 9, 9, 128, 3, 3, 64, 1, "SAME"),           # v2: BN=64 tiles, dgrad Ncol=128
    (2, 8, 8, 192, 1, 1, 320, 1, "VALID"),         # v2: N tail (320 = 2.5 x 128)
]


@pytest.mark.parametrize("backend", ["mdtf", "mdtf2"])
@pytest.mark.parametrize("case", CONV_CASES)
def test_conv_hip_fwd_dgrad_wgrad(case, backend, monkeypatch):
    monkeypatch.setenv("MDTF_CONV", backend)
    n, h, w_, c, kh, kw, co, s, pad = case
    torch.manual_seed(5)
    x = torch.randn(n, h, w_, c)
    w = torch.randn(kh, kw, c, co) * (1.0 / (kh * kw * c) ** 0.5)
    xg = x.to(DEV).bfloat16().requires_grad_(True)
    wg = w.to(DEV).bfloat16().requires_grad_(True)
    y = ops.conv2d(xg, wg, s, pad)
    xc = x.bfloat16().float().requires_grad_(True)
    wc = w.bfloat16().float().requires_grad_(True)
    yr = ops.conv2d(xc, wc, s, pad)
    assert y.shape == yr.shape
    assert _rel(y, yr) < 1e-2
    dy = torch.randn(yr.shape)
    y.backward(dy.to(DEV).bfloat16())
    yr.backward(dy.bfloat16().float())
    assert _rel(xg.grad, xc.grad) < 2e-2
    assert _rel(wg.grad, wc.grad) < 2e-2


def test_conv_hip_exact_integers(monkeypatch):
    """Small-integer data: bf16 products/sums are exact, so outputs must match bit for bit."""
    monkeypatch.setenv("MDTF_CONV", "mdtf")
    torch.manual_seed(6)
    x = torch.randint(-3, 4, (2, 10, 10, 16)).float()
    w = torch.randint(-2, 3, (3, 3, 16, 64)).float()
    y = ops.conv2d(x.to(DEV).bfloat16(), w.to(DEV).bfloat16(), 1, "SAME")
    yr = ops.conv2d(x, w, 1, "SAME")
    assert torch.equal(y.float().cpu(), yr)


def test_conv_transpose_hip(monkeypatch):
    monkeypatch.setenv("MDTF_CONV", "mdtf")
    torch.manual_seed(7)
    x = torch.randn(2, 8, 8, 32)
    w = torch.randn(3, 3, 16, 32) * 0.1                 # [kh, kw, cout, cin]
    xg = x.to(DEV).bfloat16().requires_grad_(True)
    wg = w.to(DEV).bfloat16().requires_grad_(True)
    y = ops.conv2d_transpose(xg, wg, [2, 16, 16, 16], 2, "SAME")
    xc = x.bfloat16().float().requires_grad_(True)
    wc = w.bfloat16().float().requires_grad_(True)
    yr = ops.conv2d_transpose(xc, wc, [2, 16, 16, 16], 2, "SAME")
    assert _rel(y, yr) < 1e-2
    dy = torch.randn(yr.shape)
    y.backward(dy.to(DEV).bfloat16())
    yr.backward(dy.bfloat16().float())
    assert _rel(xg.grad, xc.grad) < 2e-2
    assert _rel(wg.grad, wc.grad) < 2e-2


def _one_step(dev, dtype, x, y, depth=50, blocks=None, grads=False):
    import mdtf
    from mdtf.models import ResNet, SoftmaxCrossEntropyLoss
    from mdtf.runtime import Net, Tower
    from mdtf.train import step as S
    from mdtf.train import variables as V
    V.reset_default_graph()
    S.reset()
    store = V.get_store()
    store.device = torch.device(dev)
    store.compute_dtype = dtype
    store.generator.manual_seed(123)
    xp = mdtf.placeholder(torch.float32, [None] + list(x.shape[1:]))
    yp = mdtf.placeholder(torch.int64, [None])
    opt = mdtf.train.GradientDescentOptimizer(0.1)
    tg = []
    model = ResNet(depth, num_classes=16, zero_init_residual=False)
    if blocks is not None:
        model.blocks = blocks                    # a shallower net of the same bottleneck / BN / kernel structure
    tower = Tower(Net(model), "tower_0/", tg, xp, yp, SoftmaxCrossEntropyLoss(), opt, batch_size=x.shape[0])
    _, loss, _ = tower.process()
    op = opt.apply_gradients(Tower.average_gradients(tg), global_step=mdtf.train.get_or_create_global_step())
    sess = mdtf.train.MonitoredTrainingSession(log_step_count_steps=0)
    before = {v.name: v.master.detach().float().cpu().clone() for v in store.trainable_variables()}
    _, lv = sess.run([op, loss], feed_dict={xp: x, yp: y})
    if grads:
        return float(lv), {v.name: v.grad.detach().float().cpu().clone() for v in store.trainable_variables()}
    after = {v.name: v.master.detach().float().cpu().clone() for v in store.trainable_variables()}
    return float(lv), before, after


def test_resnet50_step_loss_matches_cpu_fp32_reference(monkeypatch):
    """ResNet-50 training step (fused conv+BN, pooling, dense, xent) vs the fp32 CPU engine: the loss
    within 4 %, and EVERY gradient tensor within max(5 %, 1.5 x the error of the same step on stock
    PyTorch bf16 ops) -- at batch 16 a random-init 50-layer net's deep gradients differ from fp32 by tens
    of percent under any bf16 implementation, so stock bf16 is the yardstick."""
    torch.manual_seed(9)
    x = torch.randn(16, 64, 64, 3)
    y = torch.randint(0, 16, (16,))
    l_cpu, g_cpu = _one_step("cpu", None, x, y, grads=True)
    l_gpu, g_gpu = _one_step(DEV, torch.bfloat16, x, y, grads=True)
    monkeypatch.setenv("MDTF_KERNELS", "torch")
    l_stk, g_stk = _one_step(DEV, torch.bfloat16, x, y, grads=True)
    monkeypatch.setenv("MDTF_KERNELS", "native")
    # the loss of this random-init 50-layer net (no zero-init residual, batch-16 BN statistics over 64 values
    # in stage 4) is chaotic in bf16: stock PyTorch bf16 lands 0.3-1.4 % from fp32 on different runs of the
    # same step, and rounding the shortcut BN output or not (ops.bn.DeferredBN) moves ours by 2 %; the
    # shallower nets of the stage-1 test hold 0.5 %.  The per-gradient checks below are the strict ones.
    assert abs(l_cpu - l_gpu) / abs(l_cpu) < 4e-2, (l_cpu, l_gpu, l_stk)
    assert len(g_cpu) > 150
    _check_grads({k: (_rel(g_gpu[k], g_cpu[k]), _rel(g_stk[k], g_cpu[k])) for k in g_cpu})


def _check_grads(errs):
    """errs: name -> (mdtf bf16 relative error, stock bf16 relative error) vs fp32.  Per tensor: within
    5 %, or within 1.5x of stock (near-cancelling BN sums are noise-dominated for both, and atomics make
    either run's rounding order vary); over the tensors where bf16 itself exceeds 5 %: the median
    mdtf/stock ratio below 1.1."""
    ratios = []
    for k, (e, e_stock) in errs.items():
        assert e < max(0.05, 1.5 * e_stock), (k, e, e_stock)
        if e_stock > 0.05:
            ratios.append(e / e_stock)
    if ratios:
        assert sorted(ratios)[len(ratios) // 2] < 1.1, sorted(ratios)


def test_resnet_stage1_every_gradient_matches_cpu_fp32(monkeypatch):
    """Every gradient tensor (each conv weight, BN gamma/beta, the dense layer) of a ResNet-v1.5 with
    the full stage 1 (3 bottleneck units incl. the projection shortcut) and the first stage-2 unit
    (strided 3x3, strided projection), batch 16: GPU bf16 (mdtf kernels) vs the fp32 CPU engine, next
    to the same step on stock PyTorch bf16 ops (MDTF_KERNELS=torch: MIOpen / hipBLASLt) as the measure
    of what bf16 itself costs.  Each mdtf gradient must be within 5 % of fp32, or no worse than 1.5x
    the stock bf16 error for tensors where bf16 alone exceeds that (BN parameters of layers followed by
    another BN get gradients that nearly cancel over the batch), and the median mdtf/stock error ratio
    over those tensors must stay below 1.1."""
    torch.manual_seed(5)
    x = torch.randn(16, 64, 64, 3)
    y = torch.randint(0, 16, (16,))
    l_cpu, g_cpu = _one_step("cpu", None, x, y, blocks=[3, 1], grads=True)
    l_gpu, g_gpu = _one_step(DEV, torch.bfloat16, x, y, blocks=[3, 1], grads=True)
    monkeypatch.setenv("MDTF_KERNELS", "torch")
    l_stk, g_stk = _one_step(DEV, torch.bfloat16, x, y, blocks=[3, 1], grads=True)
    monkeypatch.setenv("MDTF_KERNELS", "native")
    assert abs(l_cpu - l_gpu) / abs(l_cpu) < 5e-3, (l_cpu, l_gpu)
    errs = {k: (_rel(g_gpu[k], g_cpu[k]), _rel(g_stk[k], g_cpu[k])) for k in g_cpu}
    worst = sorted(errs.items(), key=lambda kv: -kv[1][0])[:8]
    print("worst relative gradient errors (mdtf, stock bf16):", worst)
    assert len(errs) > 40
    _check_grads(errs)


def test_resnet_projection_dgrad_fused_into_conv1(monkeypatch):
    """The strided projection's data gradient deferred in the block input's sink and fused with conv1's
    (mdtf_conv_ws_dual, one pass) == the two data gradients run one after the other (MDTF_DUAL_DGRAD=0): same
    loss, every gradient as close to the fp32 CPU step; the fused path must actually run (stage-2 unit 1)."""
    from mdtf.models import resnet
    from mdtf.ops import conv as C
    monkeypatch.setattr(resnet, "PROJ_LATE", True)
    torch.manual_seed(7)
    x = torch.randn(8, 64, 64, 3)
    y = torch.randint(0, 16, (8,))
    n0 = C.DUAL_FUSED[0]
    lf, gf = _one_step(DEV, torch.bfloat16, x, y, blocks=[1, 1], grads=True)
    assert C.DUAL_FUSED[0] > n0
    monkeypatch.setattr(C, "DUAL_DGRAD", False)
    lo, go = _one_step(DEV, torch.bfloat16, x, y, blocks=[1, 1], grads=True)
    assert lf == lo
    # the fused pass rounds the summed gradient once (the unfused one rounds the first contribution to bf16
    # before accumulating): compare both against fp32; BN parameters whose gradients nearly cancel over the
    # batch amplify either rounding, so the bound is relative to the unfused error there
    lc, gc = _one_step("cpu", None, x, y, blocks=[1, 1], grads=True)
    _check_grads({k: (_rel(gf[k], gc[k]), _rel(go[k], gc[k])) for k in gc})


class _Tiny(object):
    """conv-BN-ReLU, max-pool, bottleneck-style residual pair, GAP, dense."""

    def inference(self, x):
        from mdtf.layers import tools
        from mdtf.train import variables as V
        store = V.get_store()
        if store.compute_dtype is not None:
            x = x.to(store.compute_dtype)
        x = tools.conv_bn("c1", x, 64, 3, 1, relu=True)
        x = ops.max_pool(x, 3, 2, "SAME")
        s = x
        y = tools.conv_bn("c2", x, 64, 1, 1, relu=True)
        x = tools.conv_bn("c3", y, 64, 3, 1, relu=True, residual=s)
        x = tools.conv_bn("c4", x, 128, 3, 2, relu=True)
        x = ops.global_avg_pool(x)
        return tools.dense("logits", x, 16)


def _tiny_step(dev, dt, x, y):
    import mdtf
    from mdtf.models import SoftmaxCrossEntropyLoss
    from mdtf.runtime import Model, Net, Tower
    from mdtf.train import step as S
    from mdtf.train import variables as V
    V.reset_default_graph()
    S.reset()
    store = V.get_store()
    store.device = torch.device(dev)
    store.compute_dtype = dt
    store.generator.manual_seed(123)
    xp = mdtf.placeholder(torch.float32, [None] + list(x.shape[1:]))
    yp = mdtf.placeholder(torch.int64, [None])
    opt = mdtf.train.GradientDescentOptimizer(0.1)
    tg = []
    M = type("TinyModel", (_Tiny, Model), {})
    t = Tower(Net(M()), "tower_0/", tg, xp, yp, SoftmaxCrossEntropyLoss(), opt, batch_size=x.shape[0])
    _, loss, _ = t.process()
    op = opt.apply_gradients(Tower.average_gradients(tg), global_step=mdtf.train.get_or_create_global_step())
    sess = mdtf.train.MonitoredTrainingSession(log_step_count_steps=0)
    _, lv = sess.run([op, loss], feed_dict={xp: x, yp: y})
    return float(lv), {v.name: v.grad.detach().float().cpu().clone() for v in store.trainable_variables()}


@pytest.mark.parametrize("conv_backend", ["mdtf", "miopen"])
def test_engine_step_matches_cpu_fp32_reference(conv_backend, monkeypatch):
    """Full engine step on the GPU kernels (fused conv->BN stats, fp32 grad sinks, fused SGD) vs fp32 CPU."""
    monkeypatch.setenv("MDTF_CONV", conv_backend)
    torch.manual_seed(0)
    x = torch.randn(32, 16, 16, 8)
    y = torch.randint(0, 16, (32,))
    lc, gc = _tiny_step("cpu", None, x, y)
    lg, gg = _tiny_step(DEV, torch.bfloat16, x, y)
    monkeypatch.setenv("MDTF_KERNELS", "torch")
    _, gs = _tiny_step(DEV, torch.bfloat16, x, y)
    monkeypatch.setenv("MDTF_KERNELS", "native")
    assert abs(lc - lg) / lc < 5e-3
    for k in gc:
        e, e_stock = _rel(gg[k], gc[k]), _rel(gs[k], gc[k])
        assert e < max(0.05, 1.5 * e_stock), (k, e, e_stock)    # (was: every gradient within 15 %)


@pytest.mark.parametrize("shape,k,s,co,relu,res", [((8, 14, 14, 64), 3, 1, 64, True, False),
                                                   ((8, 14, 14, 64), 1, 1, 256, True, True),
                                                   ((4, 16, 16, 128), 3, 2, 128, False, False)])
def test_conv_bn_fused_stats(shape, k, s, co, relu, res, monkeypatch):
    """conv epilogue BN statistics + finalize/apply vs the fp32 reference (fwd + grads)."""
    monkeypatch.setenv("MDTF_CONV", "mdtf")
    torch.manual_seed(10)
    x = torch.randn(shape)
    w = torch.randn(k, k, shape[-1], co) * (1.0 / (k * k * shape[-1]) ** 0.5)
    g = torch.rand(co) + 0.5
    b = torch.randn(co) * 0.1
    pad = "SAME" if s == 1 else ((k - 1) // 2, (k - 1) // 2)
    r0 = torch.randn(shape[0], shape[1] // s, shape[2] // s, co)
    outs = {}
    for dev, dt in ((DEV, torch.bfloat16), ("cpu", torch.float32)):
        xx = x.to(dev).to(dt).requires_grad_(True)
        ww = w.to(dev).to(dt).requires_grad_(True)
        gg = g.to(dev).requires_grad_(True)
        bb = b.to(dev).requires_grad_(True)
        mm = torch.zeros(co, device=dev)
        mv = torch.ones(co, device=dev)
        oh = shape[1] // s
        rr = r0.to(dev).to(dt).requires_grad_(True) if res else None
        y = ops.conv_bn(xx, ww, gg, bb, mm, mv, s, pad, True, 0.9, 1e-5, relu, rr)
        dy = torch.randn(y.shape, generator=torch.Generator().manual_seed(1)).to(dev).to(dt)
        y.backward(dy)
        outs[dev] = dict(y=y.detach(), dx=xx.grad, dw=ww.grad, dg=gg.grad, db=bb.grad, mm=mm, mv=mv,
                         dr=rr.grad if res else None)
    for key in ("y", "dx", "dw", "dg", "db", "mm", "mv"):
        assert _rel(outs[DEV][key], outs["cpu"][key]) < 5e-2, key
    if res:
        assert _rel(outs[DEV]["dr"], outs["cpu"]["dr"]) < 5e-2


@pytest.mark.parametrize("path", ["fused", "pos_bcast", "gather"])
def test_bert_embeddings_fused_vs_fp32(path, monkeypatch):
    """word[ids] + pos[s] + type[types] vs fp32 lookups on the CPU: output and the three table gradients.  fused:
    one kernel each way (csrc/transformer.hip); pos_bcast: three-op path with the position rows added by broadcast
    and their gradient a column sum over the batch (the step's default); gather: position ids looked up."""
    from mdtf.ops import transformer as T
    monkeypatch.setattr(T, "BERT_EMBED_FUSED", path == "fused")
    monkeypatch.setattr(T, "POS_BCAST", path == "pos_bcast")
    torch.manual_seed(21)
    B, S_, H, Vv = 12, 24, 64, 50
    word, pos, typ = torch.randn(Vv, H), torch.randn(40, H), torch.randn(2, H)
    ids = torch.randint(0, Vv, (B, S_))
    types = torch.randint(0, 2, (B, S_))
    dy = torch.randn(B, S_, H)
    outs = {}
    for dev, dt in ((DEV, torch.bfloat16), ("cpu", torch.float32)):
        ts = [t.to(dev).to(dt).requires_grad_(True) for t in (word, pos, typ)]
        y = T.bert_embeddings(ts[0], ts[1], ts[2], ids.to(dev), types.to(dev))
        y.backward(dy.to(dev).to(dt))
        outs[dev] = [y.detach()] + [t.grad for t in ts]
    for a, r in zip(outs[DEV], outs["cpu"]):
        assert _rel(a, r) < 2e-2


@pytest.mark.parametrize("zero_gamma", [False, True, "tiny"])
def test_stem_bn_backward_statistics_from_pooled_tensors(zero_gamma, monkeypatch):
    """The fused stem's BN backward statistics from the pooled tensors (csrc/bn.hip maxpool_bn_bwd_reduce_pooled:
    x recovered from the pooled y at each window's argmax; channels with gamma == 0, or a gamma so small beside a
    large beta that bf16 y cannot give x back, gather x instead) == the input-row pass over x: filter / gamma /
    beta gradients."""
    from mdtf.ops import bn as B
    torch.manual_seed(14)
    x = torch.randn(8, 38, 38, 3)
    w = torch.randn(7, 7, 3, 64) * (1.0 / 147 ** 0.5)
    g = torch.rand(64) + 0.5
    b = torch.randn(64) * 0.2
    if zero_gamma == "tiny":
        g[::5] = 1e-3              # |shift / scale| ~ 3000 std: bf16 y rounding would swamp x
        b[::5] = 3.0
    elif zero_gamma:
        g[::7] = 0.0
    dy0 = torch.randn(8, 10, 10, 64, generator=torch.Generator().manual_seed(5))
    outs = {}
    monkeypatch.setattr(B, "FUSED_STEM", True)
    for pooled in (True, False):
        monkeypatch.setattr(B, "STEM_POOLED_STATS", pooled)
        xx = x.to(DEV).bfloat16()
        ww = w.to(DEV).bfloat16().requires_grad_(True)
        gg = g.to(DEV).requires_grad_(True)
        bb = b.to(DEV).requires_grad_(True)
        y = ops.conv_bn(xx, ww, gg, bb, torch.zeros(64, device=DEV), torch.ones(64, device=DEV), 2, (3, 3), True,
                        0.9, 1e-5, True, None, pool=(3, 2, "SAME"))
        y.backward(dy0.to(DEV).bfloat16())
        outs[pooled] = dict(dw=ww.grad.float(), dg=gg.grad.float(), db=bb.grad.float())
    for key in ("dw", "dg", "db"):
        assert _rel(outs[True][key], outs[False][key]) < 1e-2, (key, _rel(outs[True][key], outs[False][key]))


@pytest.mark.parametrize("hw", [64, 38])
def test_stem_pool_bn_input_gradient_row_pairs(hw, monkeypatch):
    """The fused stem backward's input gradient by pairs of input rows with the pooled rows staged in LDS
    (csrc/bn.hip maxpool_bn_dx_pairs) == the per-row kernel (maxpool_bn_dx_rows): filter / gamma / beta gradients
    of the stem, even and odd conv-output sizes (first and last row pairs half outside the image)."""
    from mdtf.ops import bn as B
    from mdtf.ops import _native as N
    N.register("mdtf_bn_pool_dx_pairs", [N.I], restype=None)
    torch.manual_seed(15)
    x = torch.randn(4, hw, hw, 3)
    w = torch.randn(7, 7, 3, 64) * (1.0 / 147 ** 0.5)
    g = torch.rand(64) + 0.5
    b = torch.randn(64) * 0.2
    monkeypatch.setattr(B, "FUSED_STEM", True)
    outs = {}
    try:
        for pairs in (1, 0):
            N.fn("mdtf_bn_pool_dx_pairs")(pairs)
            ww = w.to(DEV).bfloat16().requires_grad_(True)
            gg = g.to(DEV).requires_grad_(True)
            bb = b.to(DEV).requires_grad_(True)
            y = ops.conv_bn(x.to(DEV).bfloat16(), ww, gg, bb, torch.zeros(64, device=DEV),
                            torch.ones(64, device=DEV), 2, (3, 3), True, 0.9, 1e-5, True, None, pool=(3, 2, "SAME"))
            y.backward(torch.randn(y.shape, generator=torch.Generator().manual_seed(6)).to(DEV).bfloat16())
            outs[pairs] = dict(dw=ww.grad.float(), dg=gg.grad.float(), db=bb.grad.float())
    finally:
        N.fn("mdtf_bn_pool_dx_pairs")(1)
    for key in ("dw", "dg", "db"):
        assert _rel(outs[1][key], outs[0][key]) < 1e-3, (key, _rel(outs[1][key], outs[0][key]))


def test_stem_conv_bn_relu_maxpool_fused_vs_unfused(monkeypatch):
    """ResNet stem conv 7x7/2 -> BN -> ReLU -> max pool 3x3/2 SAME: the fused BN+ReLU+pool kernels
    (csrc/bn.hip mdtf_bn_relu_maxpool_fwd / mdtf_maxpool_bn_bwd) vs the unfused GPU passes on the same bf16
    inputs (pooled output, filter / gamma / beta gradients, moving statistics), and the unfused path vs the fp32
    CPU reference (looser: bf16 vs fp32 conv outputs flip some near-tie max-pool winners)."""
    from mdtf.ops import bn as B
    calls = []
    real = B.bn_relu_maxpool_nhwc
    monkeypatch.setattr(B, "bn_relu_maxpool_nhwc", lambda *a, **k: calls.append(1) or real(*a, **k))
    torch.manual_seed(12)
    x = torch.randn(8, 38, 38, 3)
    w = torch.randn(7, 7, 3, 64) * (1.0 / 147 ** 0.5)
    g = torch.rand(64) + 0.5
    b = torch.randn(64) * 0.2
    dy0 = torch.randn(8, 10, 10, 64, generator=torch.Generator().manual_seed(3))
    outs = {}
    for name, dev, dt, fused in (("fused", DEV, torch.bfloat16, True), ("unfused", DEV, torch.bfloat16, False),
                                 ("cpu", "cpu", torch.float32, False)):
        monkeypatch.setattr(B, "FUSED_STEM", fused)
        xx = x.to(dev).to(dt).requires_grad_(True)
        ww = w.to(dev).to(dt).requires_grad_(True)
        gg = g.to(dev).requires_grad_(True)
        bb = b.to(dev).requires_grad_(True)
        mm = torch.zeros(64, device=dev)
        mv = torch.ones(64, device=dev)
        y = ops.conv_bn(xx, ww, gg, bb, mm, mv, 2, (3, 3), True, 0.9, 1e-5, True, None, pool=(3, 2, "SAME"))
        assert tuple(y.shape) == (8, 10, 10, 64)
        y.backward(dy0.to(dev).to(dt))
        outs[name] = dict(y=y.detach(), dw=ww.grad, dg=gg.grad, db=bb.grad, mm=mm, mv=mv)
    assert calls == [1]
    assert _rel(outs["fused"]["y"], outs["unfused"]["y"]) < 1e-2
    for key in ("y", "dw", "dg", "db", "mm", "mv"):
        # the fused backward keeps the pooled gradient in fp32 up to the BN (the unfused path rounds it to bf16
        # first): it must be at least as close to the fp32 reference as the unfused path
        e_f, e_u = _rel(outs["fused"][key], outs["cpu"][key]), _rel(outs["unfused"][key], outs["cpu"][key])
        assert e_u < 1e-1 and e_f <= 1.3 * e_u + 1e-2, (key, e_f, e_u)


@pytest.mark.parametrize("H,res,rows", [(768, True, 37), (1024, False, 37), (64, True, 37), (256, True, 37),
                                        (768, False, 4099)])
def test_layernorm_kernel(H, res, rows):
    """Forward + backward vs fp32 CPU: a wave per row (1024, 64) and 32 lanes per row (768 = 3 x 32 vectors,
    256 = 1 x 32), odd row counts (partial blocks, half-filled waves)."""
    from mdtf.ops import transformer as T
    torch.manual_seed(11)
    x = torch.randn(rows, H) * 2 + 1
    r = torch.randn(rows, H) if res else None
    g = torch.rand(H) + 0.5
    b = torch.randn(H)
    outs = {}
    for dev, dt in ((DEV, torch.bfloat16), ("cpu", torch.float32)):
        xx = x.to(dev).to(dt).requires_grad_(True)
        rr = r.to(dev).to(dt).requires_grad_(True) if res else None
        gg = g.to(dev).requires_grad_(True)
        bb = b.to(dev).requires_grad_(True)
        y = T.layer_norm(xx, gg, bb, 1e-12, residual=rr)
        y.backward(torch.randn(rows, H, generator=torch.Generator().manual_seed(2)).to(dev).to(dt))
        outs[dev] = (y.detach(), xx.grad, gg.grad, bb.grad, rr.grad if res else None)
    for i in range(4):
        assert _rel(outs[DEV][i], outs["cpu"][i]) < 2e-2, i
    if res:
        assert _rel(outs[DEV][4], outs["cpu"][4]) < 2e-2


@pytest.mark.parametrize("cols", [128, 512, 40])
def test_masked_softmax_kernel(cols):
    from mdtf.ops import transformer as T
    torch.manual_seed(12)
    x = torch.randn(2, 3, 5, cols) * 4
    mask = (torch.rand(2, cols) < 0.2).float() * -10000.0
    outs = {}
    for dev, dt in ((DEV, torch.bfloat16), ("cpu", torch.float32)):
        xx = x.to(dev).to(dt).requires_grad_(True)
        y = T.masked_softmax(xx, mask.to(dev), 0.125)
        y.backward(torch.randn(x.shape, generator=torch.Generator().manual_seed(3)).to(dev).to(dt))
        outs[dev] = (y.detach(), xx.grad)
    assert _rel(outs[DEV][0], outs["cpu"][0]) < 1e-2
    assert _rel(outs[DEV][1], outs["cpu"][1]) < 2e-2


@pytest.mark.parametrize("vocab,B,S,H", [(100, 7, 9, 64), (2, 64, 128, 768), (3, 5, 33, 1024)])
def test_embedding_kernel(vocab, B, S, H):
    """vocab <= 4 (token types) takes the per-block partial-sum backward instead of per-element atomics."""
    from mdtf.ops import transformer as T
    torch.manual_seed(13)
    table = torch.randn(vocab, H)
    ids = torch.randint(0, vocab, (B, S))
    outs = {}
    for dev, dt in ((DEV, torch.bfloat16), ("cpu", torch.float32)):
        tt = table.to(dev).to(dt).requires_grad_(True)
        y = T.embedding_lookup(tt, ids.to(dev))
        y.backward(torch.randn(B, S, H, generator=torch.Generator().manual_seed(4)).to(dev).to(dt))
        outs[dev] = (y.detach(), tt.grad)
    assert _rel(outs[DEV][0], outs["cpu"][0]) < 1e-2
    assert _rel(outs[DEV][1], outs["cpu"][1]) < 2e-2


def test_bert_tiny_train_step_gpu():
    import mdtf
    from mdtf.models import Bert, BertPretrainingLoss, SyntheticBertLoader
    from mdtf.runtime import Net, Tower
    from mdtf.train import variables as V
    store = V.get_store()
    store.device = torch.device(DEV)
    store.compute_dtype = torch.bfloat16
    ld = SyntheticBertLoader(seq_len=32, max_predictions=5, vocab=1000)
    ld.batch_size = 8
    raw, gt = ld.load_train_batch()
    opt = mdtf.train.AdamWeightDecayOptimizer(1e-3)
    tg = []
    t = Tower(Net(Bert("tiny", vocab_size=1000, seq_len=32, max_predictions=5, dropout=0.0)), "tower_0/", tg, raw, gt,
              BertPretrainingLoss(5), opt, batch_size=8)
    _, loss, _ = t.process()
    op = opt.apply_gradients(Tower.average_gradients(tg), global_step=mdtf.train.get_or_create_global_step())
    sess = mdtf.train.MonitoredTrainingSession(log_step_count_steps=0)
    ls = []
    for _ in range(20):
        _, l = sess.run([op, loss])
        ls.append(float(l))
    assert ls[-1] < 0.5 * ls[0], ls


def test_grad_store_first_matches_zero_and_accumulate(monkeypatch):
    """Store-first gradient slots (train/variables.py claim_store, parallel/flat.py zero_grad(skip_stored)): the
    weight-gradient kernel overwrites the slots it is the only writer of, and those slots are left out of the next
    step's zero fill (one multi-range fill launch).  Tiny BERT over 4096 tokens so the dense weight gradients run on
    csrc/gemm_wg.hip: losses and final gradients equal the zero-then-accumulate path."""
    import mdtf
    from mdtf.models import Bert, BertPretrainingLoss, SyntheticBertLoader
    from mdtf.runtime import Net, Tower
    from mdtf.train import step as S
    from mdtf.train import variables as V
    monkeypatch.setenv("MDTF_WG_SQUARE", "1")          # the tiny widths on the weight-gradient kernel
    runs = {}
    for on in (True, False):
        monkeypatch.setattr(V, "STORE_FIRST", on)
        V.reset_default_graph()
        S.reset()
        store = V.get_store()
        store.device = torch.device(DEV)
        store.compute_dtype = torch.bfloat16
        store.generator.manual_seed(7)
        ld = SyntheticBertLoader(seq_len=32, max_predictions=5, vocab=512, seed=3)
        ld.batch_size = 128
        raw, gt = ld.load_train_batch()
        opt = mdtf.train.GradientDescentOptimizer(0.05)
        tg = []
        t = Tower(Net(Bert("tiny", vocab_size=512, seq_len=32, max_predictions=5, dropout=0.0)), "tower_0/", tg, raw,
                  gt, BertPretrainingLoss(5), opt, batch_size=128)
        _, loss, _ = t.process()
        op = opt.apply_gradients(Tower.average_gradients(tg), global_step=mdtf.train.get_or_create_global_step())
        sess = mdtf.train.MonitoredTrainingSession(log_step_count_steps=0)
        ls = [float(sess.run([op, loss])[1]) for _ in range(4)]
        vs = store.trainable_variables()
        runs[on] = (ls, {v.name: v.grad.detach().float().cpu().clone() for v in vs},
                    {v.name for v in vs if getattr(v, "skip_zero", False)})
    assert runs[True][2], "no gradient slot was store-written and skipped by the zero fill"
    assert not runs[False][2]
    assert runs[True][0] == runs[False][0], (runs[True][0], runs[False][0])
    for k, g in runs[False][1].items():
        # store-written slots are 0 + x == x bitwise; fp32 atomics (the tied embedding's scatter-add onto the
        # decoder's stored gradient, bias sums) add in an order that differs run to run
        assert torch.allclose(runs[True][1][k], g, rtol=1e-4, atol=1e-6), k


def test_fill_ranges_zero():
    """csrc/kernels.hip fill_ranges_kernel: zeroes exactly the given ranges (odd starts / lengths, float4 and
    scalar paths, ranges across 4096-element block boundaries)."""
    from mdtf.ops import _native as N
    if "mdtf_fill_ranges_zero" not in N.SIGNATURES:
        N.register("mdtf_fill_ranges_zero", [N.P, N.P, N.I, N.L, N.P])
    buf = torch.arange(1, 20001, dtype=torch.float32, device=DEV)
    ranges = [(0, 3), (5, 4100), (4105, 1), (5000, 7), (9001, 6000), (19999, 1)]
    rt = torch.tensor([x for r in ranges for x in r], dtype=torch.int64, device=DEV)
    N.check(N.fn("mdtf_fill_ranges_zero")(N.ptr(buf), N.ptr(rt), len(ranges), sum(n for _, n in ranges),
                                           N.stream_ptr()), "fill")
    ref = torch.arange(1, 20001, dtype=torch.float32)
    for o, n in ranges:
        ref[o:o + n] = 0
    assert torch.equal(buf.cpu(), ref)


def test_weight_cat_cache_matches_torch_cat(monkeypatch):
    """q|k|v weight concatenations refreshed by one batched copy per step (ops.gemm._WeightCats) train exactly like
    a torch.cat per layer: same losses over several steps (the weights change every step)."""
    import mdtf
    from mdtf.models import Bert, BertPretrainingLoss, SyntheticBertLoader
    from mdtf.ops import gemm as G
    from mdtf.runtime import Net, Tower
    from mdtf.train import step as S
    from mdtf.train import variables as V
    runs = {}
    for cache in ("1", "0"):
        monkeypatch.setenv("MDTF_WEIGHT_CAT_CACHE", cache)
        V.reset_default_graph()
        S.reset()
        store = V.get_store()
        store.device = torch.device(DEV)
        store.compute_dtype = torch.bfloat16
        store.generator.manual_seed(99)
        ld = SyntheticBertLoader(seq_len=32, max_predictions=5, vocab=512, seed=4)
        ld.batch_size = 8
        raw, gt = ld.load_train_batch()
        opt = mdtf.train.AdamWeightDecayOptimizer(1e-3)
        tg = []
        t = Tower(Net(Bert("tiny", vocab_size=512, seq_len=32, max_predictions=5, dropout=0.0)), "tower_0/", tg, raw,
                  gt, BertPretrainingLoss(5), opt, batch_size=8)
        _, loss, _ = t.process()
        op = opt.apply_gradients(Tower.average_gradients(tg), global_step=mdtf.train.get_or_create_global_step())
        sess = mdtf.train.MonitoredTrainingSession(log_step_count_steps=0)
        ls = []
        for _ in range(5):
            _, l = sess.run([op, loss])
            ls.append(float(l))
        runs[cache] = (ls, len(G._CATS.entries))
    assert runs["1"][1] > 0, "no q|k|v group was registered"
    for a, b in zip(runs["1"][0], runs["0"][0]):
        assert abs(a - b) <= 1e-3 * max(1.0, abs(b)), (runs["1"][0], runs["0"][0])


def _bert_step(dev, dt, raw, gt, seq=32, heads_dim=None, dropout=0.0):
    import mdtf
    from mdtf.models import Bert, BertPretrainingLoss
    from mdtf.runtime import Net, Tower
    from mdtf.train import step as S
    from mdtf.train import variables as V
    V.reset_default_graph()
    S.reset()
    store = V.get_store()
    store.device = torch.device(dev)
    store.compute_dtype = dt
    store.generator.manual_seed(321)
    rp = mdtf.placeholder(torch.int64, [None, raw.shape[1]])
    gp = mdtf.placeholder(torch.int64, [None, gt.shape[1]])
    opt = mdtf.train.GradientDescentOptimizer(0.1)
    tg = []
    model = Bert("tiny", vocab_size=512, seq_len=seq, max_predictions=5, dropout=dropout)
    if heads_dim:                      # tiny width, but head dim 64 (2 heads) so the fused kernel applies
        model.heads = model.H // heads_dim
    t = Tower(Net(model), "tower_0/", tg, rp, gp, BertPretrainingLoss(5), opt, batch_size=raw.shape[0])
    _, loss, _ = t.process()
    op = opt.apply_gradients(Tower.average_gradients(tg), global_step=mdtf.train.get_or_create_global_step())
    sess = mdtf.train.MonitoredTrainingSession(log_step_count_steps=0)
    _, lv = sess.run([op, loss], feed_dict={rp: raw, gp: gt})
    return float(lv), {v.name: v.grad.detach().float().cpu().clone() for v in store.trainable_variables()}


def test_bert_engine_step_matches_cpu_fp32_reference():
    """BERT step on the GPU path (fused QKV GEMM, fp32 GEMM weight-grad sinks, colsum bias grads, LN/softmax/
    embedding kernels, tied decoder) vs the fp32 CPU path: same loss, same gradients."""
    from mdtf.models import SyntheticBertLoader
    from mdtf.train import variables as V
    V.get_store().device = torch.device("cpu")
    ld = SyntheticBertLoader(seq_len=32, max_predictions=5, vocab=512, seed=3)
    ld.batch_size = 8
    raw, gt = ld._make()
    lc, gc = _bert_step("cpu", None, raw, gt)
    lg, gg = _bert_step(DEV, torch.bfloat16, raw, gt)
    assert abs(lc - lg) / lc < 1e-2, (lc, lg)
    assert len(gc) == len(gg)
    for k in gc:
        if k.endswith("key/bias"):
            # softmax is invariant to a per-row shift: d loss / d key-bias is exactly 0 (rounding noise only)
            assert float(gg[k].abs().max()) < 1e-2 * float(gc[k.replace("key", "query")].abs().max()) + 1e-4
            continue
        assert _rel(gg[k], gc[k]) < 0.1, (k, _rel(gg[k], gc[k]))


@pytest.mark.parametrize("M,C", [(8192, 768), (1000, 3072), (37, 64), (50, 10)])
def test_colsum_kernel(M, C):
    from mdtf.ops import kernels as K
    x = torch.randn(M, C)
    out = torch.ones(C, device=DEV)
    K.colsum_into(x.to(DEV).bfloat16(), out)
    ref = x.bfloat16().float().sum(0) + 1
    assert _rel(out.cpu(), ref) < 1e-4


@pytest.mark.parametrize("B,R,S", [(2, 72, 200), (1, 4608, 512), (3, 8, 64)])
def test_transpose16(B, R, S):
    from mdtf.ops import kernels
    x = torch.randn(B, R, S).bfloat16()
    y = kernels.transpose_brs(x.to(DEV), B, R, S)
    assert torch.equal(y.cpu(), x.transpose(1, 2))


def test_conv_stats_buffer_reuse(monkeypatch):
    """Back-to-back fused conv->BN layers share the persistent, kernel-re-zeroed statistics buffer."""
    monkeypatch.setenv("MDTF_CONV", "mdtf2")
    torch.manual_seed(9)
    x = torch.randn(4, 8, 8, 64)
    ws = [torch.randn(3, 3, 64, 64) * 0.05 for _ in range(3)]
    outs = {}
    for dev, dt in ((DEV, torch.bfloat16), ("cpu", torch.float32)):
        h = x.to(dev).to(dt)
        for w in ws:
            g = torch.ones(64, device=dev)
            b = torch.zeros(64, device=dev)
            h = ops.conv_bn(h, w.to(dev).to(dt), g, b, torch.zeros(64, device=dev), torch.ones(64, device=dev),
                            strides=1, padding="SAME", relu=True)
        outs[dev] = h.float().cpu()
    assert _rel(outs[DEV], outs["cpu"]) < 3e-2


def _attn_keep_mask(seed, B, nh, S, p):
    """Reproduce csrc/attention.hip's dropout keep bits (hash of (bh, q, k) and the seed)."""
    import numpy as np
    idx = np.arange(B * nh * S * S, dtype=np.uint64).astype(np.uint32)
    x = (idx * np.uint32(0x9E3779B1)) ^ np.uint32(seed)
    x ^= x >> np.uint32(16)
    x = x * np.uint32(0x7feb352d)
    x ^= x >> np.uint32(15)
    x = x * np.uint32(0x846ca68b)
    x ^= x >> np.uint32(16)
    thr = np.uint32(min(int(p * 4294967296.0), 4294967295))
    return torch.from_numpy((x >= thr).reshape(B, nh, S, S))


@pytest.mark.parametrize("p_drop", [0.0, 0.1])
@pytest.mark.parametrize("B,S,nh,dh,flash", [(3, 128, 4, 64, False), (3, 128, 4, 64, True), (2, 384, 3, 64, True),
                                              (1, 512, 2, 64, True), (2, 256, 2, 128, True), (1, 512, 2, 128, True),
                                              (2, 192, 3, 64, True), (1, 320, 2, 128, True), (2, 64, 2, 64, True)])
def test_fused_attention_fwd_bwd(p_drop, B, S, nh, dh, flash, monkeypatch):
    """Fused attention (S = 128 whole-sequence kernels, or the tiled online-softmax kernels for any
    S % 64 == 0 -- 192 / 320 end on a half query block -- and head dim 64 / 128) forward and backward vs fp32
    with the same dropout bits."""
    from mdtf.ops import transformer as T
    monkeypatch.setattr(T, "FLASH_ALWAYS", flash)
    torch.manual_seed(21 + S + dh)
    H = nh * dh
    qkv = torch.randn(B * S, 3 * H) * 0.5
    mask = (torch.rand(B, S) < 0.15).float() * -10000.0
    seed = 1234567
    dout = torch.randn(B * S, H)
    # kernel
    xg = qkv.to(DEV).bfloat16().requires_grad_(True)
    out = T._FusedAttention.apply(xg, mask.to(DEV), B, S, nh, p_drop, seed)
    out.backward(dout.to(DEV).bfloat16())
    # fp32 reference with the same dropout bits
    xr = qkv.bfloat16().float().requires_grad_(True)
    q, k, v = xr.reshape(B, S, 3, nh, dh).unbind(2)
    q, k, v = q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2)
    s = q @ k.transpose(-1, -2) / dh ** 0.5 + mask[:, None, None, :]
    pr = torch.softmax(s, -1)
    if p_drop:
        keep = _attn_keep_mask(T.effective_seed(seed, xg.device), B, nh, S, p_drop)
        pr = pr * keep / (1 - p_drop)
    ref = (pr @ v).transpose(1, 2).reshape(B * S, H)
    ref.backward(dout.bfloat16().float())
    assert _rel(out, ref) < 1.5e-2
    g, gr = xg.grad.float().cpu(), xr.grad
    for part in range(3):      # dq, dk, dv
        sl = slice(part * H, (part + 1) * H)
        assert _rel(g[:, sl], gr[:, sl]) < 3e-2, part


@pytest.mark.parametrize("p_drop", [0.0, 0.1])
def test_attention_bwd_v2_matches_v1(p_drop):
    """S = 128 attention backward: the register-resident v2 kernel (two workgroups per CU, S and dP recomputed
    per phase) gives the same dQ/dK/dV as the v1 kernel with [q][k] LDS images, with and without dropout."""
    from mdtf.ops import _native as NN
    from mdtf.ops import transformer as T
    torch.manual_seed(33)
    B, S_, nh, dh = 5, 128, 12, 64
    H = nh * dh
    qkv = (torch.randn(B * S_, 3 * H, device=DEV) * 0.5).bfloat16()
    mask = ((torch.rand(B, S_, device=DEV) < 0.2).float() * -10000.0)
    dout = torch.randn(B * S_, H, device=DEV).bfloat16()
    grads = []
    prev = NN.fn("mdtf_set_attn_bwd")(2)
    try:
        for v in (2, 1):
            NN.fn("mdtf_set_attn_bwd")(v)
            x = qkv.clone().requires_grad_(True)
            T._FusedAttention.apply(x, mask, B, S_, nh, p_drop, 777).backward(dout)
            grads.append(x.grad.float())
    finally:
        NN.fn("mdtf_set_attn_bwd")(prev)
    for part in range(3):
        sl = slice(part * H, (part + 1) * H)
        assert _rel(grads[0][:, sl], grads[1][:, sl]) < 1e-2, part


@pytest.mark.parametrize("p_drop", [0.0, 0.1])
def test_attention_bwd_split_phases_match_v2(p_drop):
    """S = 128 attention backward with the two phases as separate workgroups (csrc/attention.hip attn_bwd_v2s,
    MDTF_ATTN_BWD=v2s): the same arithmetic per output element as attn_bwd_v2, so dQ / dK / dV are bitwise equal,
    with and without dropout (and the key mask)."""
    from mdtf.ops import _native as NN
    from mdtf.ops import transformer as T
    torch.manual_seed(35)
    B, S_, nh, dh = 3, 128, 12, 64
    H = nh * dh
    qkv = (torch.randn(B * S_, 3 * H, device=DEV) * 0.5).bfloat16()
    mask = ((torch.rand(B, S_, device=DEV) < 0.2).float() * -10000.0)
    dout = torch.randn(B * S_, H, device=DEV).bfloat16()
    grads = []
    prev = NN.fn("mdtf_set_attn_bwd")(3)
    try:
        for v in (3, 2):
            NN.fn("mdtf_set_attn_bwd")(v)
            x = qkv.clone().requires_grad_(True)
            T._FusedAttention.apply(x, mask, B, S_, nh, p_drop, 778).backward(dout)
            grads.append(x.grad.float())
    finally:
        NN.fn("mdtf_set_attn_bwd")(prev)
    assert torch.equal(grads[0], grads[1])


@pytest.mark.parametrize("p_drop", [0.0, 0.1])
@pytest.mark.parametrize("grid", [7, 1])
def test_attention_persistent_matches_per_item(p_drop, grid):
    """S = 128 attention: the persistent kernels (csrc/attention.hip attn_fwd_pp / attn_bwd_pp: one workgroup walks
    several (batch, head) items with the next item's operands DMA'd into the other half of a double buffer) give the
    per-item kernels' context, logsumexp-consistent backward and dQ/dK/dV.  grid 7 over 60 items: 8-9 items per
    workgroup (both buffers, an uneven tail); grid 1 (the value 1 means one workgroup per CU): one item each."""
    from mdtf.ops import _native as NN
    from mdtf.ops import transformer as T
    torch.manual_seed(34)
    B, S_, nh, dh = 5, 128, 12, 64
    H = nh * dh
    qkv = (torch.randn(B * S_, 3 * H, device=DEV) * 0.5).bfloat16()
    mask = ((torch.rand(B, S_, device=DEV) < 0.2).float() * -10000.0)
    dout = torch.randn(B * S_, H, device=DEV).bfloat16()
    res = []
    prev = NN.fn("mdtf_set_attn_pp")(0)
    try:
        for pp in (0, grid):
            NN.fn("mdtf_set_attn_pp")(pp)
            x = qkv.clone().requires_grad_(True)
            out = T._FusedAttention.apply(x, mask, B, S_, nh, p_drop, 4242)
            out.backward(dout)
            torch.cuda.synchronize()
            res.append((out.float(), x.grad.float()))
    finally:
        NN.fn("mdtf_set_attn_pp")(prev)
    assert torch.equal(res[0][0], res[1][0])          # same arithmetic per element in both forward forms
    for part in range(3):
        sl = slice(part * H, (part + 1) * H)
        assert _rel(res[1][1][:, sl], res[0][1][:, sl]) < 1e-2, part


def test_bert_fused_vs_unfused_attention_path(monkeypatch):
    """BERT step: fused-attention kernel path == unfused matmul/softmax path (same weights, no dropout)."""
    from mdtf.models import SyntheticBertLoader
    from mdtf.ops import transformer as T
    from mdtf.train import variables as V
    V.get_store().device = torch.device("cpu")
    ld = SyntheticBertLoader(seq_len=128, max_predictions=5, vocab=512, seed=4)
    ld.batch_size = 4
    raw, gt = ld._make()

    def run(fused):
        monkeypatch.setattr(T, "FUSED_SEQ", 128 if fused else -1)
        return _bert_step(DEV, torch.bfloat16, raw, gt, seq=128, heads_dim=64)
    lf, gf = run(True)
    lu, gu = run(False)
    assert abs(lf - lu) / lu < 1e-2
    for k in gf:
        if k.endswith("key/bias"):
            continue
        assert _rel(gf[k], gu[k]) < 0.1, (k, _rel(gf[k], gu[k]))


def test_bert_activation_sinks_match_autograd(monkeypatch):
    """BERT step with dropout: LayerNorm outputs as gradient sinks (d(residual) handed to the sink, the
    next dense layer's dgrad accumulating into it inside its GEMM, fused q|k|v bias column sum) == the
    same step with plain autograd gradient adds."""
    from mdtf.models import SyntheticBertLoader
    from mdtf.ops import actsink
    from mdtf.train import variables as V
    V.get_store().device = torch.device("cpu")
    ld = SyntheticBertLoader(seq_len=128, max_predictions=5, vocab=512, seed=5)
    ld.batch_size = 4
    raw, gt = ld._make()
    out = {}
    for enabled in (True, False):
        monkeypatch.setattr(actsink, "ENABLED", enabled)
        torch.manual_seed(11)                        # same dropout masks in both runs
        out[enabled] = _bert_step(DEV, torch.bfloat16, raw, gt, seq=128, heads_dim=64, dropout=0.1)
    (ls, gs), (la, ga) = out[True], out[False]
    assert abs(ls - la) / la < 1e-3
    for k in ga:
        if k.endswith("key/bias"):                   # zero up to rounding (softmax is shift invariant)
            continue
        assert _rel(gs[k], ga[k]) < 2e-2, (k, _rel(gs[k], ga[k]))


def test_deterministic_mode_bitwise_repeatable():
    """MDTF deterministic mode: two identical engine steps give bit-identical gradients
    (BN statistics rows per M tile, unsplit weight-gradient GEMMs, fixed-order reductions)."""
    from mdtf.ops import _native
    torch.manual_seed(0)
    x = torch.randn(32, 16, 16, 64)
    y = torch.randint(0, 16, (32,))
    _native.set_deterministic(True)
    try:
        l1, g1 = _tiny_step(DEV, torch.bfloat16, x, y)
        l2, g2 = _tiny_step(DEV, torch.bfloat16, x, y)
    finally:
        _native.set_deterministic(False)
    assert l1 == l2
    for k in g1:
        assert torch.equal(g1[k], g2[k]), k
    from mdtf.models import SyntheticBertLoader
    from mdtf.train import variables as V
    V.get_store().device = torch.device("cpu")
    ld = SyntheticBertLoader(seq_len=32, max_predictions=5, vocab=512, seed=3)
    ld.batch_size = 8
    raw, gt = ld._make()
    _native.set_deterministic(True)
    try:
        b1 = _bert_step(DEV, torch.bfloat16, raw, gt)
        b2 = _bert_step(DEV, torch.bfloat16, raw, gt)
    finally:
        _native.set_deterministic(False)
    assert b1[0] == b2[0]
    for k in b1[1]:
        assert torch.equal(b1[1][k], b2[1][k]), k


@pytest.mark.parametrize("M,K,N,col0,ld", [(8192, 768, 768, 768, 2304), (1000, 128, 192, 0, 192), (64, 64, 64, 64, 256)])
def test_gemm_wgrad_into_strided(M, K, N, col0, ld):
    from mdtf.ops import gemm
    torch.manual_seed(31)
    x = torch.randn(M, K, device=DEV).bfloat16()
    dfull = torch.randn(M, ld, device=DEV).bfloat16()
    d = dfull[:, col0:col0 + N]
    out = torch.full((K, N), 0.5, device=DEV)
    gemm.wgrad_into(out, x, d)
    ref = x.float().t() @ d.float() + 0.5
    assert _rel(out, ref) < 1e-4


@pytest.mark.parametrize("M,K,N,col0,ld,det", [(8192, 768, 768, 768, 2304, False), (8192, 768, 3072, 0, 3072, False),
                                               (1000, 128, 192, 0, 192, False), (2048, 192, 128, 64, 256, True)])
def test_gemm_wgrad_fused_bias(M, K, N, col0, ld, det):
    """The weight-gradient kernel also adds the column sums of d (the bias gradient) into dbias."""
    from mdtf.ops import _native, gemm
    torch.manual_seed(37)
    x = torch.randn(M, K, device=DEV).bfloat16()
    d = torch.randn(M, ld, device=DEV).bfloat16()[:, col0:col0 + N]
    out = torch.full((K, N), 0.25, device=DEV)
    db = torch.full((N,), -1.0, device=DEV)
    _native.set_deterministic(det)
    try:
        fused = gemm.wgrad_into(out, x, d, db)
    finally:
        _native.set_deterministic(False)
    assert fused
    assert _rel(out, x.float().t() @ d.float() + 0.25) < 1e-4
    assert _rel(db, d.float().sum(0) - 1.0) < 1e-4


def _hash_keep(seed, n, p):
    import numpy as np
    idx = np.arange(n, dtype=np.uint64).astype(np.uint32)
    x = (idx * np.uint32(0x9E3779B1)) ^ np.uint32(seed)
    x ^= x >> np.uint32(16)
    x = x * np.uint32(0x7feb352d)
    x ^= x >> np.uint32(15)
    x = x * np.uint32(0x846ca68b)
    x ^= x >> np.uint32(16)
    return torch.from_numpy(x >= np.uint32(min(int(p * 4294967296.0), 4294967295)))


def test_layernorm_fused_dropout():
    from mdtf.ops import transformer as T
    torch.manual_seed(41)
    rows, H, p, seed = 300, 768, 0.1, 987654
    x = torch.randn(rows, H)
    r = torch.randn(rows, H)
    g = torch.rand(H) + 0.5
    b = torch.randn(H)
    dy = torch.randn(rows, H)
    xg = x.to(DEV).bfloat16().requires_grad_(True)
    rg = r.to(DEV).bfloat16().requires_grad_(True)
    y = T._LayerNorm.apply(xg, rg, g.to(DEV), b.to(DEV), 1e-12, p, seed)
    y.backward(dy.to(DEV).bfloat16())
    keep = _hash_keep(T.effective_seed(seed, xg.device), rows * H, p).view(rows, H).float()
    xc = x.bfloat16().float().requires_grad_(True)
    rc = r.bfloat16().float().requires_grad_(True)
    s = xc * keep / (1 - p) + rc
    yr = torch.nn.functional.layer_norm(s, (H,), g, b, 1e-12)
    yr.backward(dy.bfloat16().float())
    assert _rel(y, yr) < 2e-2
    assert _rel(xg.grad, xc.grad) < 2e-2
    assert _rel(rg.grad, rc.grad) < 2e-2


@pytest.mark.parametrize("stages", [1, 2, 3])
def test_conv_v2_stages_k64(stages):
    """v2 forward/dgrad with a single K step (1x1 conv, 64 channels) at every pipeline depth."""
    from mdtf.ops import conv as C
    torch.manual_seed(17)
    x = torch.randn(4, 10, 10, 64, device=DEV).bfloat16()
    w = (torch.randn(1, 1, 64, 192, device=DEV) * 0.1).bfloat16()
    y = C.mdtf_fwd(x, w, (10, 10), (1, 1), (0, 0, 0, 0), (1, 1), 128, 64, None, 2, stages)
    ref = (x.float().reshape(-1, 64) @ w.float().reshape(64, 192)).reshape(4, 10, 10, 192)
    assert _rel(y, ref) < 1e-2
    dy = torch.randn(4, 10, 10, 64, device=DEV).bfloat16()
    w2 = (torch.randn(1, 1, 192, 64, device=DEV) * 0.1).bfloat16()
    dx = C.mdtf_dgrad(dy, w2, (4, 10, 10, 192), (1, 1), (0, 0, 0, 0), (1, 1), 128, 64, 2, stages)
    ref = (dy.float().reshape(-1, 64) @ w2.float().reshape(192, 64).t()).reshape(4, 10, 10, 192)
    assert _rel(dx, ref) < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("k,s,h,w,pads", [(3, 2, 15, 14, (1, 1, 1, 1)), (1, 2, 14, 14, (0, 0, 0, 0)),
                                          (3, 2, 8, 9, (0, 1, 0, 1)), (4, 3, 13, 11, (1, 2, 1, 1)),
                                          (7, 2, 16, 16, (3, 3, 3, 3))])
@pytest.mark.parametrize("stages", [1, 2, 3])
def test_conv_v2_strided_dgrad(k, s, h, w, pads, stages):
    """Strided dgrad on the v2 kernel, one launch per stride-parity class (classes without taps write
    zeros), plain and accumulating, vs the fp32 autograd reference."""
    from mdtf.ops import conv as C
    torch.manual_seed(k * 100 + h)
    n, c, co = 2, 72, 128
    oh = (h + pads[0] + pads[1] - k) // s + 1
    ow = (w + pads[2] + pads[3] - k) // s + 1
    wt = (torch.randn(k, k, c, co) / (k * k * c) ** 0.5).bfloat16()
    dy = torch.randn(n, oh, ow, co).bfloat16()
    xr = torch.zeros(n, c, h, w, requires_grad=True)
    yr = torch.nn.functional.conv2d(torch.nn.functional.pad(xr, (pads[2], pads[3], pads[0], pads[1])),
                                    wt.float().permute(3, 2, 0, 1), stride=s)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    ref = xr.grad.permute(0, 2, 3, 1)
    dx = C.mdtf_dgrad(dy.to(DEV), wt.to(DEV), (n, h, w, c), (s, s), pads, (1, 1), 64, 64, 2, stages)
    assert _rel(dx, ref) < 1e-2
    base = torch.randn(n, h, w, c).bfloat16()
    out = base.to(DEV).clone()
    C.mdtf_dgrad(dy.to(DEV), wt.to(DEV), (n, h, w, c), (s, s), pads, (1, 1), 128, 128, 2, stages, out=out,
                 accumulate=True)
    assert _rel(out, ref + base.float()) < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("stages", [1, 2])
@pytest.mark.parametrize("k,s,pad,c,co", [(3, 1, 1, 64, 128), (1, 1, 0, 128, 256), (3, 2, 1, 128, 128),
                                          (1, 2, 0, 64, 128)])
def test_conv_v2_448_row_tile(stages, k, s, pad, c, co):
    """The 448 x 128 8-wave tile (0.875-wave tile counts at ResNet shapes): forward with the BN-statistics epilogue
    and (strided) data gradient vs fp32; row counts that leave a partial 448-row tile."""
    from mdtf.ops import conv as C
    # a one-stage ring takes K == 64 only (the strided dgrad launcher adapts per class by itself)
    stages_fwd = 2 if (stages == 1 and k * k * c > 64) else stages
    torch.manual_seed(k + c + s)
    n, h, w = 3, 19, 17
    x = torch.randn(n, h, w, c, device=DEV).bfloat16()
    wt = (torch.randn(k, k, c, co, device=DEV) / (k * k * c) ** 0.5).bfloat16()
    oh, ow = (h + 2 * pad - k) // s + 1, (w + 2 * pad - k) // s + 1
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wt.float().permute(3, 2, 0, 1), stride=s,
                                     padding=pad).permute(0, 2, 3, 1)
    st = torch.zeros(2, 8, co, device=DEV)
    y = C.mdtf_fwd(x, wt, (oh, ow), (s, s), (pad,) * 4, (1, 1), 448, 128, (st[0], st[1]), 3, stages_fwd)
    assert _rel(y, ref) < 1e-2
    assert _rel(st[0].sum(0), ref.sum((0, 1, 2))) < 1e-3
    dy = torch.randn(n, oh, ow, co, device=DEV).bfloat16()
    xr = torch.zeros(n, c, h, w, device=DEV, requires_grad=True)
    torch.nn.functional.conv2d(xr, wt.float().permute(3, 2, 0, 1), stride=s, padding=pad).backward(
        dy.float().permute(0, 3, 1, 2))
    dstages = 2 if (s == 1 and k * k * co > 64 and stages == 1) else stages
    dx = C.mdtf_dgrad(dy, wt, (n, h, w, c), (s, s), (pad,) * 4, (1, 1), 448, 128, 3, dstages)
    assert _rel(dx, xr.grad.permute(0, 2, 3, 1)) < 1e-2


@pytest.mark.gpu
@pytest.mark.parametrize("bm,bn,ver,stages", [(256, 256, 3, 32), (256, 128, 3, 32), (256, 128, 3, 42),
                                              (128, 256, 3, 32), (128, 256, 3, 42), (128, 128, 2, 32),
                                              (64, 128, 2, 32), (64, 128, 2, 42)])
@pytest.mark.parametrize("k,s,pad,c,co", [(1, 1, 0, 64, 128), (1, 1, 0, 128, 256), (1, 1, 0, 192, 128),
                                          (1, 1, 0, 256, 192), (3, 1, 1, 64, 128), (1, 1, 0, 448, 128),
                                          (3, 2, 1, 128, 128), (1, 2, 0, 64, 256)])
def test_conv_v2_split_ring(bm, bn, ver, stages, k, s, pad, c, co):
    """Split A/B LDS rings (stage code 10 SA + SB: SA A stages, SB filter stages): every K-step count from 1 to 9
    (the counted vmcnt waits of the prologue / steady state / tail), forward with BN statistics, stride-1 and
    strided data gradients with the accumulate + BN-backward-statistics epilogue, vs fp32."""
    from mdtf.ops import conv as C
    torch.manual_seed(k * 7 + c + co + s)
    n, h, w = 3, 13, 11
    x = torch.randn(n, h, w, c, device=DEV).bfloat16()
    wt = (torch.randn(k, k, c, co, device=DEV) / (k * k * c) ** 0.5).bfloat16()
    oh, ow = (h + 2 * pad - k) // s + 1, (w + 2 * pad - k) // s + 1
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wt.float().permute(3, 2, 0, 1), stride=s,
                                     padding=pad).permute(0, 2, 3, 1)
    st = torch.zeros(2, 8, co, device=DEV)
    y = C.mdtf_fwd(x, wt, (oh, ow), (s, s), (pad,) * 4, (1, 1), bm, bn, (st[0], st[1]), ver, stages)
    assert _rel(y, ref) < 1e-2
    assert _rel(st[0].sum(0), ref.sum((0, 1, 2))) < 1e-3
    assert _rel(st[1].sum(0), (ref.bfloat16().float() ** 2).sum((0, 1, 2))) < 1e-2
    dy = torch.randn(n, oh, ow, co, device=DEV).bfloat16()
    xr = torch.zeros(n, c, h, w, device=DEV, requires_grad=True)
    torch.nn.functional.conv2d(xr, wt.float().permute(3, 2, 0, 1), stride=s, padding=pad).backward(
        dy.float().permute(0, 3, 1, 2))
    gref = xr.grad.permute(0, 2, 3, 1)
    dx = C.mdtf_dgrad(dy, wt, (n, h, w, c), (s, s), (pad,) * 4, (1, 1), bm, bn, ver, stages)
    assert _rel(dx, gref) < 1e-2
    # accumulate onto a base + the BN-backward statistics of the completed gradient
    base = torch.randn(n, h, w, c, device=DEV).bfloat16()
    out = base.clone()
    bx = torch.randn(n, h, w, c, device=DEV).bfloat16()
    ps = torch.zeros(2, 4, c, device=DEV)
    C.mdtf_dgrad(dy, wt, (n, h, w, c), (s, s), (pad,) * 4, (1, 1), bm, bn, ver, stages, out=out, accumulate=True,
                 bn_stats=(bx, None, ps[0], ps[1], 4))
    full = gref + base.float()
    assert _rel(out, full) < 1e-2
    g = out.float()
    assert _rel(ps[0].sum(0), g.sum((0, 1, 2))) < 1e-2
    assert _rel(ps[1].sum(0), (g * bx.float()).sum((0, 1, 2))) < 1e-2


@pytest.mark.parametrize("stages", [2, 32])
@pytest.mark.parametrize("tail", ["1", "0"])
def test_conv_v2_tail_split(stages, tail, monkeypatch):
    """The tile-count tail split of the 8-wave 256-row tiles (launch_fd_v2): 272 = 256 + 16 tiles of 256 x 256 run
    as one launch of 256 tiles + the last 4096 rows on 128 x 128 tiles.  Forward with BN statistics and data
    gradient with accumulate + BN-backward statistics vs fp32, with the split on (MDTF_CONV_TAIL=1) and off (default
    is read once per process: the other mode runs in a child)."""
    if tail == "1":
        import subprocess
        import sys
        code = ("import torch, tests.test_kernels_gpu as t; t.setup_module(None); "
                "t._tail_case(%d)" % stages)
        env = dict(__import__("os").environ, MDTF_CONV_TAIL="1")
        r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300,
                           cwd=__import__("os").path.dirname(__import__("os").path.dirname(__file__)))
        assert r.returncode == 0, r.stderr[-2000:]
        return
    _tail_case(stages)


def _tail_case(stages):
    from mdtf.ops import conv as C
    torch.manual_seed(stages)
    n, h, w, c, co = 68, 32, 32, 64, 256                      # M = 69632 rows = 272 tiles of 256
    x = torch.randn(n, h, w, c, device=DEV).bfloat16()
    wt = (torch.randn(1, 1, c, co, device=DEV) / c ** 0.5).bfloat16()
    ref = (x.float().reshape(-1, c) @ wt.float().reshape(c, co)).reshape(n, h, w, co)
    st = torch.zeros(2, 64, co, device=DEV)
    y = C.mdtf_fwd(x, wt, (h, w), (1, 1), (0, 0, 0, 0), (1, 1), 256, 256, (st[0], st[1]), 3, stages)
    assert _rel(y, ref) < 1e-2
    assert _rel(st[0].sum(0), ref.sum((0, 1, 2))) < 1e-3
    dy = torch.randn(n, h, w, c, device=DEV).bfloat16()       # dgrad of a 1x1 256 -> 64 conv: DX has 256 channels
    w2 = (torch.randn(1, 1, co, c, device=DEV) / co ** 0.5).bfloat16()
    gref = (dy.float().reshape(-1, c) @ w2.float().reshape(co, c).t()).reshape(n, h, w, co)
    base = torch.randn(n, h, w, co, device=DEV).bfloat16()
    out = base.clone()
    bx = torch.randn(n, h, w, co, device=DEV).bfloat16()
    ps = torch.zeros(2, 4, co, device=DEV)
    C.mdtf_dgrad(dy, w2, (n, h, w, co), (1, 1), (0, 0, 0, 0), (1, 1), 256, 256, 3, stages, out=out, accumulate=True,
                 bn_stats=(bx, None, ps[0], ps[1], 4))
    assert _rel(out, gref + base.float()) < 1e-2
    g = out.float()
    assert _rel(ps[0].sum(0), g.sum((0, 1, 2))) < 1e-2
    assert _rel(ps[1].sum(0), (g * bx.float()).sum((0, 1, 2))) < 1e-2


def _bits(b):
    """bool [..., C] -> the kernels' 1-bit-per-element mask bytes (element 8i + k = bit k of byte i)."""
    w = (1 << torch.arange(8, device=b.device)).to(torch.int32)
    return (b.reshape(-1, 8).to(torch.int32) * w).sum(-1).to(torch.uint8)


@pytest.mark.gpu
@pytest.mark.parametrize("c", [64, 256])
@pytest.mark.parametrize("mode", ["plain", "acc_src_stats"])
def test_strided_dgrad_zero_tap_classes_streamed(c, mode):
    """1x1 stride-2 dgrad: 3 of the 4 stride-parity classes have no filter taps.  Their pixels are written by
    one streaming launch (csrc/conv_igemm.hip dgrad_zero_classes), with the masked accumulate source and the
    BN-backward statistics (sum g*mask, sum g*mask*x) of every pixel, vs an fp32 reference."""
    from mdtf.ops import conv as C
    torch.manual_seed(c)
    n, h, w, co = 4, 14, 14, 128
    wt = (torch.randn(1, 1, c, co, device=DEV) / c ** 0.5).bfloat16()
    dy = torch.randn(n, 7, 7, co, device=DEV).bfloat16()
    ref = torch.zeros(n, h, w, c, device=DEV)
    ref[:, ::2, ::2] = (dy.float().reshape(-1, co) @ wt.float().reshape(c, co).t()).reshape(n, 7, 7, c)
    if mode == "plain":
        dx = C.mdtf_dgrad(dy, wt, (n, h, w, c), (2, 2), (0, 0, 0, 0), (1, 1), 64, 128, 2, 2)
        assert _rel(dx, ref) < 1e-2
        assert dx.float()[:, 1::2].abs().max().item() == 0 and dx.float()[:, :, 1::2].abs().max().item() == 0
        return
    g = torch.randn(n, h, w, c, device=DEV).bfloat16()
    gm = torch.rand(n, h, w, c, device=DEV) > 0.3
    x = torch.randn(n, h, w, c, device=DEV).bfloat16()
    xm = torch.rand(n, h, w, c, device=DEV) > 0.5
    slots = 4
    ps = torch.zeros(2, slots, c, device=DEV)
    out = torch.empty(n, h, w, c, device=DEV, dtype=torch.bfloat16)
    C.mdtf_dgrad(dy, wt, (n, h, w, c), (2, 2), (0, 0, 0, 0), (1, 1), 64, 128, 2, 2, out=out,
                 bn_stats=(x, _bits(xm), ps[0], ps[1], slots), acc_src=(g, _bits(gm)))
    full = ref + g.float() * gm
    assert _rel(out, full) < 1e-2
    o = out.float() * xm
    assert _rel(ps[0].sum(0), o.sum((0, 1, 2))) < 1e-3
    assert _rel(ps[1].sum(0), (o * x.float()).sum((0, 1, 2))) < 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("k,s,pad,c,co", [(3, 1, 1, 64, 192), (3, 2, 1, 128, 64), (1, 2, 0, 256, 512),
                                          (1, 1, 0, 64, 256), (5, 1, 2, 64, 64)])
def test_conv_pp_forward_with_bn_stats(tile, k, s, pad, c, co):
    """Forward conv on the ping-pong core (csrc/gemm_pp.hip mdtf_conv_pp): padding taps, strides, tile tails;
    output and the epilogue's per-channel sum y / sum y^2 vs an fp32 reference.  Every tile must accept."""
    from mdtf.ops import conv as C
    torch.manual_seed(k * 7 + s + tile)
    n, h, w = 3, 17, 15
    assert C.pp_ok("fwd", c, co, (s, s), k, k, tile)
    x = torch.randn(n, h, w, c, device=DEV).bfloat16()
    wt = (torch.randn(k, k, c, co, device=DEV) / (k * k * c) ** 0.5).bfloat16()
    oh, ow = (h + 2 * pad - k) // s + 1, (w + 2 * pad - k) // s + 1
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wt.float().permute(3, 2, 0, 1), stride=s,
                                     padding=pad).permute(0, 2, 3, 1)
    slots = 8
    st = torch.zeros(2, slots, co, device=DEV)
    y = C.pp_fwd(x, wt, (oh, ow), (s, s), (pad, pad, pad, pad), (1, 1), tile, (st[0], st[1]))
    assert y.shape == ref.shape
    assert _rel(y, ref) < 1e-2
    assert _rel(st[0].sum(0), ref.sum((0, 1, 2))) < 1e-3
    assert _rel(st[1].sum(0), (ref * ref).sum((0, 1, 2))) < 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("tile", [1, 3, 5])
@pytest.mark.parametrize("k,pad,c,co", [(3, 1, 128, 64), (1, 0, 256, 128), (3, 1, 384, 256)])
@pytest.mark.parametrize("mode", ["plain", "accumulate", "acc_src_stats"])
def test_conv_pp_dgrad(tile, k, pad, c, co, mode):
    """Stride-1 data gradient on the ping-pong core: plain, accumulating into out, and with a masked accumulate
    source + the BN-backward statistics epilogue, vs fp32.  Every listed tile must accept these shapes."""
    from mdtf.ops import conv as C
    if c % C.PP_TILES[tile][1]:
        pytest.skip("Cin not a multiple of the tile's columns (host refuses: filter rows would alias a tap)")
    torch.manual_seed(k + c + tile)
    n, h, w = 2, 13, 11
    assert C.pp_ok("dgrad", c, co, (1, 1), k, k, tile)
    wt = (torch.randn(k, k, c, co, device=DEV) / (k * k * co) ** 0.5).bfloat16()
    dy = torch.randn(n, h, w, co, device=DEV).bfloat16()
    xr = torch.zeros(n, c, h, w, device=DEV, requires_grad=True)
    yr = torch.nn.functional.conv2d(xr, wt.float().permute(3, 2, 0, 1), padding=pad)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    ref = xr.grad.permute(0, 2, 3, 1)
    if mode == "plain":
        dx = C.pp_dgrad(dy, wt, (n, h, w, c), (pad, pad, pad, pad), (1, 1), tile)
        assert _rel(dx, ref) < 1e-2
        return
    if mode == "accumulate":
        base = torch.randn(n, h, w, c, device=DEV).bfloat16()
        out = base.clone()
        C.pp_dgrad(dy, wt, (n, h, w, c), (pad, pad, pad, pad), (1, 1), tile, out=out, accumulate=True)
        assert _rel(out, ref + base.float()) < 1e-2
        return
    g = torch.randn(n, h, w, c, device=DEV).bfloat16()
    gm = torch.rand(n, h, w, c, device=DEV) > 0.3
    x = torch.randn(n, h, w, c, device=DEV).bfloat16()
    xm = torch.rand(n, h, w, c, device=DEV) > 0.5
    ps = torch.zeros(2, 4, c, device=DEV)
    out = torch.empty(n, h, w, c, device=DEV, dtype=torch.bfloat16)
    C.pp_dgrad(dy, wt, (n, h, w, c), (pad, pad, pad, pad), (1, 1), tile, out=out,
               bn_stats=(x, _bits(xm), ps[0], ps[1], 4), acc_src=(g, _bits(gm)))
    full = ref + g.float() * gm
    assert _rel(out, full) < 1e-2
    o = out.float() * xm
    assert _rel(ps[0].sum(0), o.sum((0, 1, 2))) < 1e-3
    assert _rel(ps[1].sum(0), (o * x.float()).sum((0, 1, 2))) < 1e-3


class _TinyRes(object):
    """Fan-out activations as in ResNet: a BN output feeding a conv AND a residual (identity block),
    then a block input feeding two convs (projection shortcut) -- exercises the activation-gradient sinks."""

    def inference(self, x):
        from mdtf.layers import tools
        from mdtf.train import variables as V
        store = V.get_store()
        if store.compute_dtype is not None:
            x = x.to(store.compute_dtype)
        s = tools.conv_bn("c1", x, 64, 3, 1, relu=True)
        y = tools.conv_bn("c2", s, 64, 1, 1, relu=True)
        x = tools.conv_bn("c3", y, 64, 3, 1, relu=True, residual=s)          # s: conv + identity residual
        sc = tools.conv_bn("sc", x, 128, 1, 1, relu=False)                   # x: projection conv + main conv
        z = tools.conv_bn("c4", x, 64, 1, 1, relu=True)
        x = tools.conv_bn("c5", z, 128, 3, 1, relu=True, residual=sc)
        x = ops.global_avg_pool(x)
        return tools.dense("logits", x, 16)


class _TinyStrided(object):
    """BN outputs consumed by a strided 3x3 conv, a strided 1x1 projection and stride-1 convs: the
    BN backward statistics come from stride-1 and stride-parity-class dgrad epilogues."""

    def inference(self, x):
        from mdtf.layers import tools
        from mdtf.train import variables as V
        store = V.get_store()
        if store.compute_dtype is not None:
            x = x.to(store.compute_dtype)
        s = tools.conv_bn("c1", x, 64, 3, 1, relu=True)
        y = tools.conv_bn("c2", s, 64, 3, 2, relu=True)                     # strided 3x3 dgrad -> c1 BN
        sc = tools.conv_bn("sc", s, 128, 1, 2, relu=False)                   # strided 1x1 projection -> c1 BN
        z = tools.conv_bn("c3", y, 128, 1, 1, relu=True, residual=sc)
        x = ops.global_avg_pool(z)
        return tools.dense("logits", x, 16)


@pytest.mark.parametrize("model", ["res", "strided"])
def test_bn_backward_stats_from_dgrad_epilogue(model, monkeypatch):
    """BN backward with Σdy·mask, Σdy·mask·x emitted by the completing v2 dgrad's epilogue == the
    separate reduction pass; the fused path must actually run."""
    from mdtf.ops import bn as B, conv as C
    monkeypatch.setenv("MDTF_CONV", "mdtf2")
    global _Tiny
    saved = _Tiny
    _Tiny = _TinyRes if model == "res" else _TinyStrided
    try:
        torch.manual_seed(4)
        x = torch.randn(16, 12, 12, 64)
        y = torch.randint(0, 16, (16,))
        n0 = B.FUSED_BWD[0]
        lf, gf = _tiny_step(DEV, torch.bfloat16, x, y)
        assert B.FUSED_BWD[0] - n0 >= 2
        monkeypatch.setattr(C, "BWD_STATS", False)
        lo, go = _tiny_step(DEV, torch.bfloat16, x, y)
    finally:
        _Tiny = saved
    assert lf == lo
    for k in go:
        assert _rel(gf[k], go[k]) < 1e-2, (k, _rel(gf[k], go[k]))


class _TinyDual(object):
    """A projection-shortcut block as ResNet builds it: the shortcut BN deferred into the residual BN
    (relu(BN(x) + BN2(r)), ops.bn.DeferredBN); ``stride`` 2 makes both the shortcut and the 3x3 strided."""
    stride = 1

    def inference(self, x):
        from mdtf.layers import tools
        from mdtf.train import variables as V
        store = V.get_store()
        if store.compute_dtype is not None:
            x = x.to(store.compute_dtype)
        s = tools.conv_bn("c1", x, 64, 3, 1, relu=True)
        sc = tools.conv_bn("sc", s, 128, 1, self.stride, relu=False, defer=True)
        z = tools.conv_bn("c2", s, 64, 1, 1, relu=True)
        z = tools.conv_bn("c3", z, 64, 3, self.stride, relu=True)
        x = tools.conv_bn("c4", z, 128, 1, 1, relu=True, residual=sc)
        x = ops.global_avg_pool(x)
        return tools.dense("logits", x, 16)


class _TinyDualStrided(_TinyDual):
    stride = 2


@pytest.mark.parametrize("model", ["res", "strided"])
def test_dual_bn_backward_one_pass_matches_two(model, monkeypatch):
    """relu(BN(x) + BN2(r)) backward: both input gradients in one pass (mdtf_bn_bwd_dual, with the main BN's
    statistics from the dgrad epilogue) == the two bn_dx passes; the one-pass kernel must actually run."""
    from mdtf.ops import bn as B
    global _Tiny
    saved = _Tiny
    _Tiny = _TinyDual if model == "res" else _TinyDualStrided
    try:
        torch.manual_seed(6)
        x = torch.randn(16, 12, 12, 64)
        y = torch.randint(0, 16, (16,))
        monkeypatch.setattr(B, "DUAL_FUSED", True)
        n0 = B.DUAL_BWD[0]
        lf, gf = _tiny_step(DEV, torch.bfloat16, x, y)
        assert B.DUAL_BWD[0] - n0 >= 1
        monkeypatch.setattr(B, "DUAL_FUSED", False)
        lo, go = _tiny_step(DEV, torch.bfloat16, x, y)
    finally:
        _Tiny = saved
    assert lf == lo
    for k in go:
        assert _rel(gf[k], go[k]) < 1e-2, (k, _rel(gf[k], go[k]))


@pytest.mark.parametrize("conv_backend", ["mdtf2", "ws"])
def test_masked_residual_gradient_folded_into_dgrad(conv_backend, monkeypatch):
    """The residual BN's identity-shortcut gradient dy*mask left pending in the sink and folded into the
    completing conv dgrad's epilogue (v2 or weight-stationary kernel, masked accumulate source) ==
    writing it out and accumulating (MDTF_MASKED_RESIDUAL=0); the folded path must actually run."""
    from mdtf.ops import actsink
    if conv_backend == "mdtf2":
        monkeypatch.setenv("MDTF_CONV", "mdtf2")
    global _Tiny
    saved = _Tiny
    _Tiny = _TinyRes
    try:
        torch.manual_seed(6)
        x = torch.randn(16, 12, 12, 64)
        y = torch.randint(0, 16, (16,))
        n0 = actsink.FOLDED[0]
        lf, gf = _tiny_step(DEV, torch.bfloat16, x, y)
        assert actsink.FOLDED[0] > n0
        monkeypatch.setattr(actsink, "MASKED_RESIDUAL", False)
        lo, go = _tiny_step(DEV, torch.bfloat16, x, y)
    finally:
        _Tiny = saved
    assert lf == lo
    for k in go:
        assert _rel(gf[k], go[k]) < 1e-2, (k, _rel(gf[k], go[k]))


@pytest.mark.parametrize("conv_backend", ["mdtf2", "miopen"])
def test_fanout_gradient_sinks(conv_backend, monkeypatch):
    """In-place fan-out gradient accumulation == autograd's add (same kernels otherwise), and both ~ fp32 CPU."""
    from mdtf.ops import actsink
    monkeypatch.setenv("MDTF_CONV", conv_backend)
    global _Tiny
    saved = _Tiny
    _Tiny = _TinyRes
    try:
        torch.manual_seed(3)
        x = torch.randn(16, 12, 12, 64)
        y = torch.randint(0, 16, (16,))
        lc, gc = _tiny_step("cpu", None, x, y)
        lg, gg = _tiny_step(DEV, torch.bfloat16, x, y)
        actsink.ENABLED = False
        try:
            lo, go = _tiny_step(DEV, torch.bfloat16, x, y)
        finally:
            actsink.ENABLED = True
    finally:
        _Tiny = saved
    assert abs(lc - lg) / lc < 5e-3 and lo == lg
    for k in gc:
        assert _rel(gg[k], go[k]) < 2e-2, (k, _rel(gg[k], go[k]))        # sinks vs autograd adds
        assert _rel(gg[k], gc[k]) < 0.25, (k, _rel(gg[k], gc[k]))        # bf16 path vs fp32 (deep-layer noise)


V3_TILES = [(256, 256, 1), (256, 256, 2), (256, 128, 1), (256, 128, 2), (256, 128, 3), (256, 64, 2),
            (256, 64, 3), (256, 64, 4), (128, 256, 2), (128, 256, 3)]


@pytest.mark.parametrize("bm,bn,stages", V3_TILES)
@pytest.mark.parametrize("geo", [(3, 9, 9, 64, 3, 320, 1), (2, 12, 12, 128, 1, 256, 1), (2, 15, 13, 64, 3, 128, 2)])
def test_conv_v2_8wave_tiles(bm, bn, stages, geo):
    """8-wave (512-thread) v2 tiles: forward with the fused BN-statistics epilogue, stride-1 / strided dgrad
    (plain and accumulating) vs fp32 references; M and N tails, one and many K steps."""
    from mdtf.ops import conv as C
    n, h, w, c, k, co, s = geo
    if stages == 1 and k * k * c > 64:
        k, s = 1, 1                                   # single-buffer tiles: one K step only
    if stages == 1:
        c = 64
    torch.manual_seed(bm + bn + stages + k)
    p = k // 2
    pads = (p, p, p, p)
    oh = (h + 2 * p - k) // s + 1
    ow = (w + 2 * p - k) // s + 1
    x = torch.randn(n, h, w, c).bfloat16()
    wt = (torch.randn(k, k, c, co) / (k * k * c) ** 0.5).bfloat16()
    xr = x.float().permute(0, 3, 1, 2)
    yr = torch.nn.functional.conv2d(xr, wt.float().permute(3, 2, 0, 1), stride=s, padding=p).permute(0, 2, 3, 1)
    sbuf = torch.zeros(2, 64, co, device=DEV)
    y = C.mdtf_fwd(x.to(DEV), wt.to(DEV), (oh, ow), (s, s), pads, (1, 1), bm, bn, (sbuf[0], sbuf[1]), 3, stages)
    assert _rel(y, yr) < 1e-2
    yf = yr.reshape(-1, co)                 # the statistics come from the fp32 accumulators
    assert _rel(sbuf[0].sum(0), yf.sum(0)) < 5e-3
    assert _rel(sbuf[1].sum(0), (yf * yf).sum(0)) < 5e-3
    if co % 64 or (stages == 1 and k * k * co > 64):
        return
    # dgrad: DX [n,h,w,c] from DY [n,oh,ow,co]; Ncol = c
    dy = torch.randn(n, oh, ow, co).bfloat16()
    xg = torch.zeros(n, c, h, w, requires_grad=True)
    yg = torch.nn.functional.conv2d(xg, wt.float().permute(3, 2, 0, 1), stride=s, padding=p)
    yg.backward(dy.float().permute(0, 3, 1, 2))
    ref = xg.grad.permute(0, 2, 3, 1)
    dx = C.mdtf_dgrad(dy.to(DEV), wt.to(DEV), (n, h, w, c), (s, s), pads, (1, 1), bm, bn, 3, stages)
    assert _rel(dx, ref) < 1e-2
    base = torch.randn(n, h, w, c).bfloat16()
    out = base.to(DEV).clone()
    C.mdtf_dgrad(dy.to(DEV), wt.to(DEV), (n, h, w, c), (s, s), pads, (1, 1), bm, bn, 3, stages, out=out,
                 accumulate=True)
    assert _rel(out, ref + base.float()) < 1e-2


@pytest.mark.parametrize("bm,bn,stages", [(256, 256, 2), (256, 128, 2), (256, 128, 3), (128, 256, 2), (128, 256, 3),
                                          (128, 128, 3), (64, 256, 3), (64, 256, 4), (256, 64, 3), (256, 64, 4)])
@pytest.mark.parametrize("geo", [(3, 9, 9, 64, 3, 320, 1), (2, 12, 12, 192, 1, 256, 1), (2, 15, 13, 64, 3, 128, 2),
                                 (2, 14, 14, 64, 1, 256, 1), (2, 14, 14, 256, 1, 64, 1)])
@pytest.mark.parametrize("slab", [True, False])
def test_conv_wgrad_8wave_tiles(bm, bn, stages, geo, slab, monkeypatch):
    """8-wave v2 weight-gradient tiles (split-K fp32 atomics) vs the fp32 autograd reference: R and Cout
    tails, pixel tails, strided 3x3."""
    from mdtf.ops import conv as C
    monkeypatch.setattr(C, "WGRAD_SLAB", slab)      # split-K partial slabs + reduction, or fp32 atomics
    n, h, w, c, k, co, s = geo
    torch.manual_seed(bm * 3 + bn + stages + k)
    p = k // 2
    pads = (p, p, p, p)
    x = torch.randn(n, h, w, c).bfloat16()
    wt = (torch.randn(k, k, c, co) / (k * k * c) ** 0.5).bfloat16()
    wr = wt.float().permute(3, 2, 0, 1).requires_grad_(True)
    yr = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wr, stride=s, padding=p)
    dy = torch.randn(yr.shape).bfloat16()
    yr.backward(dy.float())
    ref = wr.grad.permute(2, 3, 1, 0)                         # HWIO
    for sp in (0, 3):
        dw = C.mdtf_wgrad(x.to(DEV), dy.permute(0, 2, 3, 1).contiguous().to(DEV), wt.shape, (s, s), pads, (1, 1),
                          bm, bn, sp, ver=3, stages=stages)
        assert _rel(dw, ref) < 1e-2, sp


@pytest.mark.parametrize("geo", [(2, 56, 56, 256, 128, 512, 2), (3, 28, 28, 512, 256, 1024, 2), (2, 15, 13, 64, 128, 128, 2),
                                 (2, 9, 10, 128, 128, 256, 2)])
@pytest.mark.parametrize("tile", [(2, 8, 1), (2, 4, 1), (4, 8, 1)])
def test_conv_ws_dual_fanout_dgrad(geo, tile):
    """csrc/conv_ws.hip mdtf_conv_ws_dual: the gradient of a block input feeding a 1x1 / stride-1 conv and a
    1x1 / stride-2 projection, both data gradients in one GEMM (the sampled pixels first in the kernel's pixel order,
    the others skip the second k-range), plain and with the BN-backward statistics, vs the fp32 autograd sum; odd
    sizes (the projection's last row / column, unpaired last row)."""
    from mdtf.ops import conv as C
    n, h, w, c, c1, c2, s = geo
    torch.manual_seed(sum(geo) + tile[0] * tile[1])
    x = torch.zeros(n, c, h, w, requires_grad=True)
    w1 = (torch.randn(1, 1, c, c1) / c ** 0.5).bfloat16()
    w2 = (torch.randn(1, 1, c, c2) / c ** 0.5).bfloat16()
    y1 = torch.nn.functional.conv2d(x, w1.float().permute(3, 2, 0, 1))
    y2 = torch.nn.functional.conv2d(x, w2.float().permute(3, 2, 0, 1), stride=s)
    dy1 = torch.randn(y1.shape).bfloat16()
    dy2 = torch.randn(y2.shape).bfloat16()
    (y1 * dy1.float()).sum().add((y2 * dy2.float()).sum()).backward()
    ref = x.grad.permute(0, 2, 3, 1)
    d1 = dy1.permute(0, 2, 3, 1).contiguous().to(DEV)
    d2 = dy2.permute(0, 2, 3, 1).contiguous().to(DEV)
    pc = (d2, w2.to(DEV), (s, s))
    assert C.dual_ok((n, h, w, c), tuple(w1.shape), (1, 1), (0, 0, 0, 0), (1, 1), pc)
    dx = C.ws_dual(d1, w1.to(DEV), pc, (n, h, w, c), tile=tile)
    assert _rel(dx, ref) < 1e-2
    bx = torch.randn(n, h, w, c).bfloat16()
    mbits = torch.rand(n * h * w * c) > 0.4
    packed = (mbits.view(-1, 8).to(torch.int32) << torch.arange(8)).sum(1).to(torch.uint8)
    bsum = torch.zeros(2, 4, c, device=DEV)
    gd = C.ws_dual(d1, w1.to(DEV), pc, (n, h, w, c), tile=tile,
                   bn_stats=(bx.to(DEV), packed.to(DEV), bsum[0], bsum[1], 4))
    assert _rel(gd, ref) < 1e-2
    gm = gd.float().cpu().reshape(-1, c) * mbits.view(-1, c).float()
    assert _rel(bsum[0].sum(0), gm.sum(0)) < 5e-3
    assert _rel(bsum[1].sum(0), (gm * bx.float().reshape(-1, c)).sum(0)) < 5e-3


@pytest.mark.parametrize("splits", [64, 24, 9])
def test_conv_wgrad_slab_split_groups(splits, monkeypatch):
    """Slab reduction of many split-K partials for a small filter (1x1 64 -> 64: 16 float4 blocks, up to 64
    splits, uneven last split), vs the fp32 autograd reference."""
    from mdtf.ops import conv as C
    monkeypatch.setattr(C, "WGRAD_SLAB", True)
    n, h, w, c, co = 2, 56, 56, 64, 64
    torch.manual_seed(splits)
    x = torch.randn(n, h, w, c).bfloat16()
    wt = (torch.randn(1, 1, c, co) / c ** 0.5).bfloat16()
    wr = wt.float().permute(3, 2, 0, 1).requires_grad_(True)
    yr = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wr)
    dy = torch.randn(yr.shape).bfloat16()
    yr.backward(dy.float())
    ref = wr.grad.permute(2, 3, 1, 0)
    dw = C.mdtf_wgrad(x.to(DEV), dy.permute(0, 2, 3, 1).contiguous().to(DEV), wt.shape, (1, 1), (0, 0, 0, 0),
                      (1, 1), 128, 128, splits, ver=3, stages=3)
    assert _rel(dw, ref) < 1e-2


@pytest.mark.parametrize("ink", [True, False])
@pytest.mark.parametrize("geo", [(2, 14, 14, 64, 3, 128, 128, 256, 2, 3, 5),    # R = 576: partial 128-row tiles
                                 (2, 28, 28, 128, 1, 256, 256, 128, 2, 3, 7),
                                 (4, 7, 7, 256, 3, 64, 256, 64, 3, 3, 3),        # skinny 8-wave tile, Cout 64
                                 (2, 16, 16, 64, 1, 192, 128, 128, 2, 3, 4),     # Cout 192: partial column tile
                                 (2, 20, 20, 128, 3, 64, 128, 64, 2, 2, 6)])     # 4-wave tile
def test_conv_wgrad_inkernel_split_reduction(ink, geo, monkeypatch):
    """Split-K weight gradient summed in the kernel by each tile's last arriving workgroup (write-through partial
    tiles + tickets, MDTF_WGRAD_INK) vs the slab + reduction launch, both vs the fp32 autograd reference; the
    result accumulates into a non-zero gradient slot, and the tickets are left zeroed (a second launch agrees)."""
    from mdtf.ops import conv as C
    from mdtf.ops import mm
    monkeypatch.setattr(C, "WGRAD_SLAB", True)
    monkeypatch.setattr(C, "WGRAD_INK", ink)
    n, h, w, c, k, co, bm, bn, stages, ver, splits = geo
    torch.manual_seed(sum(geo))
    p = k // 2
    x = torch.randn(n, h, w, c).bfloat16()
    wt = (torch.randn(k, k, c, co) / (k * k * c) ** 0.5).bfloat16()
    wr = wt.float().permute(3, 2, 0, 1).requires_grad_(True)
    yr = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wr, padding=p)
    dy = torch.randn(yr.shape).bfloat16()
    yr.backward(dy.float())
    ref = wr.grad.permute(2, 3, 1, 0)
    base = torch.randn(k, k, c, co)
    xd, dyd = x.to(DEV), dy.permute(0, 2, 3, 1).contiguous().to(DEV)
    for rep in range(2):
        out = base.to(DEV).clone()
        C.mdtf_wgrad(xd, dyd, wt.shape, (1, 1), (p, p, p, p), (1, 1), bm, bn, splits, out=out, ver=ver,
                     stages=stages)
        assert _rel(out.cpu() - base, ref) < 1e-2, rep
    t = mm._tickets(torch.device(DEV), 4096)
    assert int(t.abs().sum()) == 0


@pytest.mark.parametrize("mode", ["slab", "atomics", "inkernel"])
def test_conv_wgrad_store_overwrites_slot(mode, monkeypatch):
    """``mdtf_wgrad(store=True)`` (the step's first writer of a gradient slot, V.claim_store) overwrites a slot
    holding stale values: the slab reduction stores its sum; the atomics / in-kernel-reduction epilogues get the slot
    zeroed first.  vs the fp32 autograd reference."""
    from mdtf.ops import conv as C
    monkeypatch.setattr(C, "WGRAD_SLAB", mode != "atomics")
    monkeypatch.setattr(C, "WGRAD_INK", mode == "inkernel")
    n, h, w, c, co = 2, 14, 14, 64, 128
    torch.manual_seed(5)
    x = torch.randn(n, h, w, c).bfloat16()
    wt = (torch.randn(3, 3, c, co) / (9 * c) ** 0.5).bfloat16()
    wr = wt.float().permute(3, 2, 0, 1).requires_grad_(True)
    yr = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wr, padding=1)
    dy = torch.randn(yr.shape).bfloat16()
    yr.backward(dy.float())
    ref = wr.grad.permute(2, 3, 1, 0)
    out = torch.full((3, 3, c, co), 7.0, device=DEV)
    C.mdtf_wgrad(x.to(DEV), dy.permute(0, 2, 3, 1).contiguous().to(DEV), wt.shape, (1, 1), (1, 1, 1, 1), (1, 1), 128,
                 128, 4, out=out, ver=3, stages=2, store=True)
    assert _rel(out.cpu(), ref) < 1e-2
    out2 = out.clone()                  # store off again: accumulates
    C.mdtf_wgrad(x.to(DEV), dy.permute(0, 2, 3, 1).contiguous().to(DEV), wt.shape, (1, 1), (1, 1, 1, 1), (1, 1), 128,
                 128, 4, out=out2, ver=3, stages=2)
    assert _rel(out2.cpu(), 2 * ref) < 1e-2


WS_TILES = [(4, 8, 1, 4), (4, 8, 2, 6), (4, 4, 1, 4), (2, 8, 1, 8), (2, 4, 2, 4), (4, 8, 4, 4)]


@pytest.mark.parametrize("tile", WS_TILES)
@pytest.mark.parametrize("geo", [(3, 9, 9, 64, 1, 256, 1), (2, 12, 11, 128, 3, 128, 1), (2, 15, 13, 64, 3, 64, 2),
                                 (4, 7, 7, 256, 1, 512, 2), (2, 6, 9, 96, 1, 128, 1)])
def test_conv_weight_stationary(tile, geo):
    """csrc/conv_ws.hip: forward (any stride, padded 3x3) with the fused BN-statistics epilogue, stride-1
    dgrad (flipped filter) plain / accumulating / with the BN-backward statistics, vs fp32 references;
    pixel tails, channel groups, persistent tile loops."""
    from mdtf.ops import conv as C
    n, h, w, c, k, co, s = geo
    tp, nw, cg, d = tile
    if co % (64 * cg) or (c % (64 * cg) and s == 1) or 64 * cg * k * k * max(c, co) * 2 > 160 * 1024:
        cg = 1
        tile = (tp, nw, 1, d)
    kf, kd = k * k * c, k * k * co                           # forward / dgrad reduction lengths
    pick = lambda kt: d if C.ws_depth_ok(kt, d) else next(x for x in (4, 3, 6, 2) if C.ws_depth_ok(kt, x))  # noqa
    tile = (tp, nw, cg, pick(kf))
    torch.manual_seed(sum(geo) + tp * nw * cg)
    p = k // 2
    pads = (p, p, p, p)
    oh = (h + 2 * p - k) // s + 1
    ow = (w + 2 * p - k) // s + 1
    x = torch.randn(n, h, w, c).bfloat16()
    wt = (torch.randn(k, k, c, co) / (k * k * c) ** 0.5).bfloat16()
    xr = x.float().permute(0, 3, 1, 2)
    yr = torch.nn.functional.conv2d(xr, wt.float().permute(3, 2, 0, 1), stride=s, padding=p).permute(0, 2, 3, 1)
    assert C.ws_ok("fwd", c, co, (s, s), k, k)
    for cap in (0, 3):                                       # default persistent grid and a tiny one (long loops)
        sbuf = torch.zeros(2, 8, co, device=DEV)
        y = C.ws_fwd(x.to(DEV), C.transpose_filter(wt.to(DEV)), k, k, (oh, ow), (s, s), pads, (1, 1), tile,
                     (sbuf[0], sbuf[1]), grid_cap=cap)
        assert _rel(y, yr) < 1e-2, cap
        yf = yr.reshape(-1, co)
        assert _rel(sbuf[0].sum(0), yf.sum(0)) < 5e-3
        assert _rel(sbuf[1].sum(0), (yf * yf).sum(0)) < 5e-3
    if s != 1 or c % (64 * cg):
        return
    dy = torch.randn(n, oh, ow, co).bfloat16()
    xg = torch.zeros(n, c, h, w, requires_grad=True)
    yg = torch.nn.functional.conv2d(xg, wt.float().permute(3, 2, 0, 1), stride=s, padding=p)
    yg.backward(dy.float().permute(0, 3, 1, 2))
    ref = xg.grad.permute(0, 2, 3, 1)
    assert C.ws_ok("dgrad", c, co, (s, s), k, k)
    tile = (tp, nw, cg, pick(kd))
    dx = C.ws_dgrad(dy.to(DEV), wt.to(DEV), (n, h, w, c), pads, (1, 1), tile)
    assert _rel(dx, ref) < 1e-2
    base = torch.randn(n, h, w, c).bfloat16()
    out = base.to(DEV).clone()
    C.ws_dgrad(dy.to(DEV), wt.to(DEV), (n, h, w, c), pads, (1, 1), tile, out=out, accumulate=True, grid_cap=5)
    assert _rel(out, ref + base.float()) < 1e-2
    # BN-backward statistics of the stored gradient: sum g*mask, sum g*mask*x
    bx = torch.randn(n, h, w, c).bfloat16()
    mbits = torch.rand(n * h * w * c) > 0.4
    packed = (mbits.view(-1, 8).to(torch.int32) << torch.arange(8)).sum(1).to(torch.uint8)
    bsum = torch.zeros(2, 4, c, device=DEV)
    tile_b = (2, nw, cg, tile[3])                          # BN-statistics epilogues: 2-subtile tiles
    gd = C.ws_dgrad(dy.to(DEV), wt.to(DEV), (n, h, w, c), pads, (1, 1), tile_b,
                    bn_stats=(bx.to(DEV), packed.to(DEV), bsum[0], bsum[1], 4))
    gm = gd.float().cpu().reshape(-1, c) * mbits.view(-1, c).float()
    assert _rel(bsum[0].sum(0), gm.sum(0)) < 5e-3
    assert _rel(bsum[1].sum(0), (gm * bx.float().reshape(-1, c)).sum(0)) < 5e-3


@pytest.mark.parametrize("n,h", [(2, 56), (3, 13)])
def test_conv3_rows(n, h):
    """csrc/conv_rows.hip (64 -> 64 channel 3x3 / stride 1 / pad 1, 56 wide): forward with the BN-statistics
    epilogue and the data gradient plain / with the BN-backward statistics (with and without a ReLU mask) vs fp32
    references; row groups past the image's last row (h = 13), persistent loops (n * 7 groups > 1 per block
    only at large n: here the tails)."""
    from mdtf.ops import conv as C
    w, c = 56, 64
    torch.manual_seed(n * h)
    pads = (1, 1, 1, 1)
    assert C.rows_ok((h, w), c, c, 3, 3, (1, 1), pads, (1, 1))
    x = torch.randn(n, h, w, c).bfloat16()
    wt = (torch.randn(3, 3, c, c) / (9 * c) ** 0.5).bfloat16()
    wr = wt.float().permute(3, 2, 0, 1)
    yr = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wr, padding=1).permute(0, 2, 3, 1)
    sbuf = torch.zeros(2, 8, c, device=DEV)
    y = C.ws_fwd(x.to(DEV), C.transpose_filter(wt.to(DEV)), 3, 3, (h, w), (1, 1), pads, (1, 1), (4, 8, 1, 3),
                 (sbuf[0], sbuf[1]))
    assert _rel(y, yr) < 1e-2
    yf = yr.reshape(-1, c)
    assert _rel(sbuf[0].sum(0), yf.sum(0)) < 5e-3
    assert _rel(sbuf[1].sum(0), (yf * yf).sum(0)) < 5e-3
    dy = torch.randn(n, h, w, c).bfloat16()
    xg = torch.zeros(n, c, h, w, requires_grad=True)
    torch.nn.functional.conv2d(xg, wr, padding=1).backward(dy.float().permute(0, 3, 1, 2))
    ref = xg.grad.permute(0, 2, 3, 1)
    dx = C.ws_dgrad(dy.to(DEV), wt.to(DEV), (n, h, w, c), pads, (1, 1), (2, 8, 1, 3))
    assert _rel(dx, ref) < 1e-2
    bx = torch.randn(n, h, w, c).bfloat16()
    mbits = torch.rand(n * h * w * c) > 0.4
    packed = (mbits.view(-1, 8).to(torch.int32) << torch.arange(8)).sum(1).to(torch.uint8)
    for mask in (packed, None):
        bsum = torch.zeros(2, 4, c, device=DEV)
        gd = C.ws_dgrad(dy.to(DEV), wt.to(DEV), (n, h, w, c), pads, (1, 1), (2, 8, 1, 3),
                        bn_stats=(bx.to(DEV), None if mask is None else mask.to(DEV), bsum[0], bsum[1], 4))
        assert _rel(gd, ref) < 1e-2
        gm = gd.float().cpu().reshape(-1, c)
        if mask is not None:
            gm = gm * mbits.view(-1, c).float()
        assert _rel(bsum[0].sum(0), gm.sum(0)) < 5e-3
        assert _rel(bsum[1].sum(0), (gm * bx.float().reshape(-1, c)).sum(0)) < 5e-3


@pytest.mark.parametrize("geo", [(2, 30, 31, 3, 7, 64, 2, 3), (3, 17, 16, 1, 5, 128, 1, 2), (2, 24, 24, 4, 3, 64, 2, 1),
                                 (1, 224, 224, 3, 7, 64, 2, 3)])
@pytest.mark.parametrize("kernel", ["rows", "ws"])
def test_stem_conv_forward(geo, kernel):
    """Few-channel stem forward (repack to a haloed 4-channel image + the row-staged kernel, or the streamed
    weight-stationary GEMM) with the fused BN-statistics epilogue vs the fp32 reference; ResNet's 7x7/2 RGB
    stem included."""
    from mdtf.ops import conv as C
    n, h, w, c, k, co, s, p = geo
    torch.manual_seed(sum(geo))
    x = torch.randn(n, h, w, c).bfloat16()
    wt = (torch.randn(k, k, c, co) / (k * k * c) ** 0.5).bfloat16()
    oh = (h + 2 * p - k) // s + 1
    ow = (w + 2 * p - k) // s + 1
    assert C.choose("fwd", x.shape, wt.shape, (s, s), (p, p, p, p), (1, 1)) == ("stem",)
    yr = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wt.float().permute(3, 2, 0, 1), stride=s,
                                    padding=p).permute(0, 2, 3, 1)
    sbuf = torch.zeros(2, 8, co, device=DEV)
    keep = []
    y = C.stem_fwd(x.to(DEV), wt.to(DEV), (oh, ow), (s, s), (p, p, p, p), (sbuf[0], sbuf[1]),
                   tile=C.STEM_TILE if kernel == "ws" else None, keep_x4=keep)
    assert y.shape == yr.shape
    assert _rel(y, yr) < 1e-2
    yf = yr.reshape(-1, co)
    assert _rel(sbuf[0].sum(0), yf.sum(0)) < 5e-3
    assert _rel(sbuf[1].sum(0), (yf * yf).sum(0)) < 5e-3
    if co != 64 or k > 8:
        return
    # weight gradient from the packed image (csrc/stem_wgrad.hip), accumulated into a non-zero slot
    dy = torch.randn(n, oh, ow, co).bfloat16()
    wr = wt.float().permute(3, 2, 0, 1).requires_grad_(True)
    torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wr, stride=s, padding=p).backward(
        dy.float().permute(0, 3, 1, 2))
    ref = wr.grad.permute(2, 3, 1, 0)
    base = torch.randn(k, k, c, co)
    for blocks in (0, 3):
        dw = base.clone().to(DEV)
        C.stem_wgrad(keep[0], dy.to(DEV), wt.shape, (s, s), out=dw, blocks=blocks)
        assert _rel(dw.cpu() - base, ref) < 1e-2, blocks


@pytest.mark.parametrize("M,K,N", [(1000, 768, 2304), (4100, 768, 768), (333, 768, 3072), (2048, 1024, 4096)])
def test_dense_dgrad_hand_kernel(M, K, N, monkeypatch):
    """Dense data gradient on the hand-written MFMA kernel (ops/gemm.py DGRAD_TILES, MDTF_DENSE_DGRAD=mdtf),
    plain and accumulating into a fanned-out input's gradient, vs fp32 matmul; M tails included."""
    from mdtf.ops import gemm as G
    monkeypatch.setattr(G, "HAND_DGRAD", True)
    torch.manual_seed(M + N)
    d = torch.randn(M, N).bfloat16()
    w = (torch.randn(K, N) * 0.05).bfloat16()
    ref = d.float() @ w.float().t()
    dx = G._hand_dgrad(d.to(DEV), w.to(DEV))
    assert dx is not None and dx.shape == (M, K)
    assert _rel(dx, ref) < 1e-2
    base = torch.randn(M, K).bfloat16()
    out = base.to(DEV).clone()
    G._hand_dgrad(d.to(DEV), w.to(DEV), out=out, accumulate=True)
    assert _rel(out, ref + base.float()) < 1e-2


@pytest.mark.parametrize("M,K,nw,nseg,act,bias,tile", [
    (1000, 768, 768, 3, 0, True, None), (4100, 768, 3072, 1, 2, True, None), (333, 3072, 768, 1, 0, True, None),
    (2048, 1024, 4096, 1, 1, False, None), (77, 64, 64, 2, 2, True, None),
    (8192, 768, 768, 3, 0, True, (256, 128, 2, 3)), (8192, 768, 3072, 1, 2, True, (256, 256, 2, 3)),
    (8192, 3072, 768, 1, 0, True, (128, 256, 3, 3)), (1280, 768, 768, 1, 0, True, (64, 128, 3, 2)),
    (4096, 768, 3072, 1, 2, True, (128, 128, 4, 2))])
def test_dense_fwd_hand_kernel(M, K, nw, nseg, act, bias, tile, monkeypatch):
    """Dense forward on the hand-written MFMA kernel (fd v2 MODE 3: W read in place N-contiguous, q|k|v column
    segments, bias on the accumulators, GELU/ReLU epilogue with the saved pre-activation) vs fp32 matmul;
    M tails, 4- and 8-wave tiles, 2-4 stage rings."""
    from mdtf.ops import gemm as G
    monkeypatch.setattr(G, "FWD_MODE", "mdtf")
    monkeypatch.setattr(G, "HAND_FWD", True)
    torch.manual_seed(M + nw + act)
    x = torch.randn(M, K).bfloat16()
    ws = [(torch.randn(K, nw) * 0.05).bfloat16() for _ in range(nseg)]
    b = (torch.randn(nw * nseg) * 0.5).bfloat16() if bias else None
    pre_ref = x.float() @ torch.cat([w.float() for w in ws], 1)
    if bias:
        pre_ref = pre_ref + b.float()
    act_ref = {0: lambda t: t, 1: torch.relu, 2: lambda t: torch.nn.functional.gelu(t, approximate="tanh")}[act]
    out = G.hand_fwd(x.to(DEV), [w.to(DEV) for w in ws], b.to(DEV) if bias else None, act, tile=tile)
    assert out is not None
    y, pre = out
    assert y.shape == (M, nw * nseg)
    assert _rel(y, act_ref(pre_ref)) < 1e-2
    if act == 2:
        assert _rel(pre, pre_ref) < 1e-2
        # the activation is applied to the stored (rounded) pre-activation, as the backward sees it
        assert _rel(y, act_ref(pre.float().cpu())) < 5e-3
    else:
        assert pre is None


@pytest.mark.parametrize("M,K,N,act,tile", [(8192, 3072, 768, 2, None), (1000, 3072, 768, 2, None),
                                             (333, 1024, 256, 1, None), (4096, 3072, 768, 2, (128, 256, 2, 3)),
                                             (4096, 768, 768, 2, (64, 128, 3, 2))])
def test_dense_dgrad_act_epilogue(M, K, N, act, tile):
    """Data gradient with the producer's activation backward in the epilogue: dx = (dy W^T) * act'(pre), vs
    fp32 (GELU tanh form / ReLU); M tails, 4- and 8-wave tiles."""
    from mdtf.ops import gemm as G
    torch.manual_seed(M + K)
    dy = torch.randn(M, N).bfloat16()
    w = (torch.randn(K, N) * 0.05).bfloat16()
    pre = (torch.randn(M, K) * 2).bfloat16()
    p = pre.float().requires_grad_()
    y = torch.nn.functional.gelu(p, approximate="tanh") if act == 2 else torch.relu(p)
    y.backward((dy.float() @ w.float().t()))
    dx = G.hand_dgrad_act(dy.to(DEV), w.to(DEV), pre.to(DEV), act, tile=tile)
    assert dx is not None and dx.shape == (M, K)
    assert _rel(dx, p.grad) < 1e-2


@pytest.mark.parametrize("engine", ["pp", "legacy"])
def test_ffn_fused_act_backward_matches_unfused(engine, monkeypatch):
    """ffn(): GELU backward fused into the second layer's data gradient gives the same gradients as the
    separate activation-backward pass (the GEMM core's act-backward epilogue, or the r2 conv-kernel MODE 4)."""
    from mdtf.ops import gemm as G
    monkeypatch.setattr(G, "PP", engine == "pp")
    monkeypatch.setattr(G, "PP_FWD", "fused")      # the core takes both FFN layers (default "act": only the first)
    torch.manual_seed(5)
    x = torch.randn(2048, 768, device=DEV).bfloat16()
    w1 = (torch.randn(768, 3072, device=DEV) * 0.03).bfloat16().requires_grad_()
    b1 = (torch.randn(3072, device=DEV) * 0.1).bfloat16().requires_grad_()
    w2 = (torch.randn(3072, 768, device=DEV) * 0.02).bfloat16().requires_grad_()
    b2 = (torch.randn(768, device=DEV) * 0.1).bfloat16().requires_grad_()
    res = []
    calls = []
    if engine == "pp":
        real = G.mm.dgrad

        def counted(*a, **k):
            out = real(*a, **k)
            if k.get("act_pre") is not None:
                calls.append(out is not None)
            return out
        monkeypatch.setattr(G.mm, "dgrad", counted)
    else:
        real = G.hand_dgrad_act

        def counted(*a, **k):
            out = real(*a, **k)
            calls.append(out is not None)
            return out
        monkeypatch.setattr(G, "hand_dgrad_act", counted)
    for fuse in (True, False):
        monkeypatch.setattr(G, "FFN_FUSE", fuse)
        xi = x.clone().requires_grad_()
        y = G.ffn(xi, w1, b1, w2, b2)
        y.float().square().mean().backward()
        res.append([y.detach(), xi.grad] + [t.grad for t in (w1, b1, w2, b2)])
        for t in (w1, b1, w2, b2):
            t.grad = None
    assert calls == [True], calls              # the fused epilogue ran once (fused pass only)
    for a, r in zip(res[0], res[1]):
        assert _rel(a, r) < 1e-2


def test_dense_layer_hand_fwd_matches_library(monkeypatch):
    """A dense layer (q|k|v segments + GELU FFN) forward and backward: the hand-written GEMM core (segments,
    bias + GELU epilogue, its data and weight gradients) vs the hipBLASLt path give the same outputs and
    gradients."""
    from mdtf.ops import gemm as G
    torch.manual_seed(3)
    x = torch.randn(512, 768, device=DEV).bfloat16()
    ws = [(torch.randn(768, 768, device=DEV) * 0.05).bfloat16().requires_grad_() for _ in range(3)]
    bs = [(torch.randn(768, device=DEV) * 0.1).bfloat16().requires_grad_() for _ in range(3)]
    w2 = (torch.randn(2304, 3072, device=DEV) * 0.02).bfloat16().requires_grad_()
    b2 = (torch.randn(3072, device=DEV) * 0.1).bfloat16().requires_grad_()
    res = []
    for hand in (True, False):
        monkeypatch.setattr(G, "PP", hand)
        for k in ("PP_FWD", "PP_DGRAD", "PP_WGRAD"):     # every product of both layers on the core
            monkeypatch.setattr(G, k, "all")
        monkeypatch.setattr(G, "HAND_FWD", False)
        monkeypatch.setattr(G, "FWD_MODE", "hipblaslt")
        xi = x.clone().requires_grad_()
        h = G.dense_multi(xi, ws, bs)
        y = G.dense(h, w2, b2, act="gelu")
        y.float().square().mean().backward()
        res.append([y.detach(), xi.grad] + [t.grad for t in ws + bs + [w2, b2]])
        for t in ws + bs + [w2, b2]:
            t.grad = None
    for a, r in zip(res[0], res[1]):
        assert _rel(a, r) < 1e-2


def _tiny_steps(steps, monkeypatch, cache):
    import mdtf
    from mdtf.models import SoftmaxCrossEntropyLoss
    from mdtf.runtime import Model, Net, Tower
    from mdtf.train import step as S
    from mdtf.train import variables as V
    monkeypatch.setenv("MDTF_FILTER_CACHE", "1" if cache else "0")
    V.reset_default_graph()
    S.reset()
    store = V.get_store()
    store.device = torch.device(DEV)
    store.compute_dtype = torch.bfloat16
    store.generator.manual_seed(123)
    torch.manual_seed(0)
    x = torch.randn(32, 16, 16, 8)
    y = torch.randint(0, 16, (32,))
    xp = mdtf.placeholder(torch.float32, [None, 16, 16, 8])
    yp = mdtf.placeholder(torch.int64, [None])
    opt = mdtf.train.MomentumOptimizer(0.1, 0.9)
    tg = []
    M = type("TinyModel", (_Tiny, Model), {})
    Tower(Net(M()), "tower_0/", tg, xp, yp, SoftmaxCrossEntropyLoss(), opt, batch_size=32).process()
    op = opt.apply_gradients(Tower.average_gradients(tg), global_step=mdtf.train.get_or_create_global_step())
    sess = mdtf.train.MonitoredTrainingSession(log_step_count_steps=0)
    for _ in range(steps):
        sess.run(op, feed_dict={xp: x, yp: y})
    return {v.name: v.master.detach().float().cpu().clone() for v in store.trainable_variables()}


def test_filter_transpose_cache_matches_per_call(monkeypatch):
    """Conv filters' K-contiguous copies refreshed by one batched kernel per step (ops/conv.py
    _FilterTransposes) give bitwise the same training as per-call transposes (deterministic mode)."""
    from mdtf.ops import conv as C
    _native.set_deterministic(True)
    try:
        monkeypatch.setenv("MDTF_CONV", "mdtf2")
        a = _tiny_steps(4, monkeypatch, True)
        assert len(C._WT.order) >= 3                 # every v2-forward filter was registered
        b = _tiny_steps(4, monkeypatch, False)
    finally:
        _native.set_deterministic(False)
    for k in a:
        assert torch.equal(a[k], b[k]), k


# ---------------------------------------------------------------------------- ping-pong GEMM core (csrc/gemm_pp.hip)
@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 5])
@pytest.mark.parametrize("M,N,K", [(1000, 768, 320), (264, 1536, 704), (4096, 768, 768), (768, 2304, 1024),
                                   (1001, 768, 3072), (257, 512, 4096)])
def test_gemm_core_three_layouts_vs_fp32(tile, M, N, K):
    """Forward (bias + GELU + saved pre-activation), data gradient (plain and accumulate) and fp32 weight
    gradient (1 and 2 K-splits) of every tile on odd row counts (1001, 257) and K in {320, 704, 768, 1024, 3072,
    4096}, vs fp32."""
    from mdtf.ops import mm
    torch.manual_seed(tile * 7 + M)
    rnd = lambda *s: (torch.rand(*s, device=DEV) * 2 - 1).bfloat16()
    x, w, b = rnd(M, K), rnd(K, N), rnd(N)
    pre = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    y = mm.fwd(x, w, biases=[b], act=2, pre=pre, tile=tile)
    # the forward declines exactly the tiles whose column width does not divide N (transposed B), no others
    assert (y is not None) == mm._valid(0, tile, M, N), (tile, M, N)
    if y is not None:
        ref = x.float() @ w.float() + b.float()
        assert _rel(pre, ref) < 1e-2
        assert _rel(y, torch.nn.functional.gelu(pre.float(), approximate="tanh")) < 1e-2
    dy, w2 = rnd(M, K), rnd(N, K)
    dx = mm.dgrad(dy, w2, tile=tile)
    assert dx is not None and _rel(dx, dy.float() @ w2.float().t()) < 1e-2
    acc0 = rnd(M, N)
    dxa = mm.dgrad(dy, w2, out=acc0.clone(), accumulate=True, tile=tile)
    assert _rel(dxa, dy.float() @ w2.float().t() + acc0.float()) < 1e-2
    xt, dyt = rnd(K, M), rnd(K, N)
    for sp in (1, 2):
        gw = torch.randn(M, N, device=DEV)
        ref = gw + xt.float().t() @ dyt.float()
        ok = mm.wgrad_into(gw, xt, dyt, tile=tile, splits=sp)
        assert ok == mm._valid(2, tile, M, N), (tile, M, N, sp)     # declines only transposed-edge straddles
        if ok:
            assert _rel(gw, ref) < 1e-4


def test_gemm_core_segments_and_fused_epilogues():
    """q|k|v-style weight segments in one launch (no concatenation): forward with bias + ReLU, data gradient with
    the activation backward, weight gradients into separate fp32 slots with the fused bias-gradient sums."""
    from mdtf.ops import mm
    torch.manual_seed(3)
    rnd = lambda *s: (torch.rand(*s, device=DEV) * 2 - 1).bfloat16()
    M, K, ns = 2048, 768, 768
    x = rnd(M, K)
    ws, bs = [rnd(K, ns) for _ in range(3)], [rnd(ns) for _ in range(3)]
    W, B = torch.cat(ws, 1).float(), torch.cat(bs).float()
    pre = torch.empty(M, 3 * ns, dtype=torch.bfloat16, device=DEV)
    y = mm.fwd(x, ws, biases=bs, act=1, pre=pre)
    assert _rel(pre, x.float() @ W + B) < 1e-2 and _rel(y, torch.relu(pre.float())) < 1e-2
    dy = rnd(M, 3 * ns)
    dx = mm.dgrad(dy, ws, act_pre=x, act_bwd=2)
    xf = x.float()
    s = torch.sigmoid(1.5957691216 * (xf + 0.044715 * xf ** 3))
    gelu_grad = s + 2 * xf * s * (1 - s) * 0.7978845608 * (1 + 0.134145 * xf ** 2)
    assert _rel(dx, (dy.float() @ W.t()) * gelu_grad) < 2e-2
    gws = [torch.zeros(K, ns, device=DEV) for _ in range(3)]
    dbs = [torch.zeros(ns, device=DEV) for _ in range(3)]
    assert mm.wgrad_into(gws, x, dy, dbs=dbs)
    assert _rel(torch.cat(gws, 1), x.float().t() @ dy.float()) < 1e-4
    assert _rel(torch.cat(dbs), dy.float().sum(0)) < 1e-4


# ------------------------------------------------------------------ weight-gradient kernel (csrc/gemm_wg.hip)
@pytest.mark.parametrize("bm,stages", [(128, 2), (128, 3), (128, -3), (128, -4), (256, 2), (256, 3), (256, -3)])
@pytest.mark.parametrize("T,K,N,nseg", [(8192, 768, 2304, 3), (4096, 3072, 768, 1), (704, 256, 384, 1),
                                        (64, 256, 128, 1)])
@pytest.mark.parametrize("splits", [1, 3, 7, -5, -37, -256])
@pytest.mark.parametrize("sk", [True, False])
def test_gemm_wg_vs_fp32(bm, stages, T, K, N, nseg, splits, sk, monkeypatch):
    """C_s (fp32) += x^T dy[:, seg s] with the fused bias column sums, every ring depth / loop variant and split
    count (slabs summed by the last arriving workgroup; splits > 1 run stream-K when sk, negative splits are
    stream-K worker counts: pieces cut at tile boundaries, uneven last worker), vs fp32; repeated launches are
    bitwise equal."""
    from mdtf.ops import mm
    if splits < 0 and not sk:
        pytest.skip("explicit stream-K worker count")
    monkeypatch.setattr(mm, "WG_SK", sk)
    if K % bm:
        pytest.skip("tile does not divide K")
    torch.manual_seed(T + K + splits)
    rnd = lambda *s: (torch.rand(*s, device=DEV) * 2 - 1).bfloat16()
    x, dy = rnd(T, K), rnd(T, N)
    ns = N // nseg
    g0 = [torch.randn(K, ns, device=DEV) for _ in range(nseg)]
    b0 = [torch.randn(ns, device=DEV) for _ in range(nseg)]
    gs, bs = [g.clone() for g in g0], [b.clone() for b in b0]
    assert mm.wg_into(gs, x, dy, dbs=bs, bm=bm, stages=stages, splits=splits)
    for s in range(nseg):
        d = dy[:, s * ns:(s + 1) * ns].float()
        assert _rel(gs[s] - g0[s], x.float().t() @ d) < 1e-4
        assert _rel(bs[s] - b0[s], d.sum(0)) < 1e-4
    gs2 = [g.clone() for g in g0]
    assert mm.wg_into(gs2, x, dy, bm=bm, stages=stages, splits=splits)
    assert all(torch.equal(gs[s], gs2[s]) for s in range(nseg))


def test_gemm_wg_column_slice_and_dense_backward_route():
    """dy read in place as a column slice of a wider tensor, and the BERT dense layers' backward taking the
    weight-gradient kernel (q|k|v segments, FFN) with gradients equal to fp32 autograd."""
    from mdtf.ops import gemm, mm
    torch.manual_seed(11)
    rnd = lambda *s: (torch.rand(*s, device=DEV) * 2 - 1).bfloat16()
    x, big = rnd(4096, 768), rnd(4096, 2304)
    d = big[:, 768:1536]
    g = torch.zeros(768, 768, device=DEV)
    assert mm.wg_into([g], x, d)
    assert _rel(g, x.float().t() @ d.float()) < 1e-4
    assert gemm.PP_WGRAD == "wg"
    calls = []
    orig = mm.wg_into

    def spy(*a, **k):
        calls.append(1)
        return orig(*a, **k)
    mm.wg_into = spy

    class _Slot(object):            # a Variable's fp32 gradient slot, as V.grad_sink sees it
        def __init__(self, shape):
            self.grad = torch.zeros(shape, device=DEV)
    try:
        xin = rnd(4096, 768).requires_grad_(True)
        ws = [(torch.randn(768, 768, device=DEV) * 0.05).bfloat16().requires_grad_(True) for _ in range(3)]
        bs = [(torch.randn(768, device=DEV) * 0.05).bfloat16().requires_grad_(True) for _ in range(3)]
        for t in ws + bs:
            t._mdtf_var = _Slot(t.shape)
        y = ops.dense_multi(xin, ws, bs)
        gy = rnd(*y.shape)
        y.backward(gy)
    finally:
        mm.wg_into = orig
    assert calls, "the dense backward did not take the weight-gradient kernel"
    xf = xin.detach().float()
    for j in range(3):
        d = gy[:, j * 768:(j + 1) * 768].float()
        assert _rel(ws[j]._mdtf_var.grad, xf.t() @ d) < 1e-4
        assert _rel(bs[j]._mdtf_var.grad, d.sum(0)) < 1e-4


def test_fused_apply_multi_matches_sequential():
    """The async parameter server's batched apply: k sequential Adam / momentum updates in one kernel pass."""
    from mdtf.ops import optim
    torch.manual_seed(5)
    for kind in ("momentum", "adam"):
        n = 4096
        w0 = torch.randn(n, device=DEV)
        grads = [torch.randn(n, device=DEV).bfloat16() for _ in range(4)]
        lrs, lrts = [0.1, 0.08, 0.06, 0.04], [0.01, 0.009, 0.008, 0.007]
        kw = dict(momentum=0.9, beta1=0.9, beta2=0.999, epsilon=1e-8, weight_decay=1e-4)
        a, s1, s2 = w0.clone(), torch.zeros(n, device=DEV), torch.zeros(n, device=DEV)
        shadow = torch.empty(n, dtype=torch.bfloat16, device=DEV)
        optim.apply_multi_(kind, a, grads, s1, s2, shadow, lrs, lrts, **kw)
        b, t1, t2 = w0.cpu(), torch.zeros(n), torch.zeros(n)
        optim.apply_multi_(kind, b, [g.cpu() for g in grads], t1, t2, None, lrs, lrts, **kw)
        assert torch.allclose(a.cpu(), b, atol=1e-5), kind
        assert torch.equal(shadow.cpu(), a.cpu().bfloat16())


def test_backup_workers_device_mask_two_ranks(tmp_path):
    """replicas_to_aggregate = 1 of 2 GPU replicas (sharing the GPU over gloo): the first finisher is chosen on the
    device from clock stamps (no store ticket, no host sync); exactly one contribution per step, equal weights."""
    import json
    import os
    import sys
    import torch.multiprocessing as mp
    sys.path.insert(0, os.path.dirname(__file__))
    import dist_helpers
    from mdtf.cluster.launcher import free_port
    mp.start_processes(dist_helpers.backup_gpu_worker, args=(2, free_port(), 5, str(tmp_path), 1), nprocs=2,
                       join=True, start_method="spawn")
    res = [json.load(open(str(tmp_path / ("rank%d.json" % r)))) for r in range(2)]
    assert all(r["device_mask"] for r in res)
    assert sum(r["contributed"] for r in res) == 5
    for k in res[0]["weights"]:
        assert torch.allclose(torch.tensor(res[0]["weights"][k]), torch.tensor(res[1]["weights"][k]), atol=1e-6)


def test_tied_decoder_padded_vocab_matches_fp32():
    """The tied MLM decoder over the zero-padded 30720-row vocabulary (forward with bias, split-K data gradient,
    weight + bias gradients into the padded fp32 slots) against fp32 PyTorch on the unpadded [30522, 768]
    shapes, with the loss on the strided logits view (kernels._Xent hands back the zero-padded gradient)."""
    from mdtf.ops import gemm, kernels
    from mdtf.parallel.flat import FlatParamSpace
    from mdtf.train import variables as V
    torch.manual_seed(11)
    Vn, H, M = 30522, 768, 1280
    wv = V.Variable("word_embeddings", torch.randn(Vn, H) * 0.05)
    bv = V.Variable("output_bias", torch.randn(Vn) * 0.1)
    wv.pad_rows = bv.pad_rows = gemm.decoder_pad_rows(Vn)
    assert Vn + wv.pad_rows == 30720
    FlatParamSpace([wv, bv], DEV, torch.bfloat16)
    for v in (wv, bv):
        v.grad.zero_()
    h = (torch.randn(M, H, device=DEV) * 0.5).bfloat16().requires_grad_(True)
    labels = torch.randint(0, Vn, (M,), device=DEV)
    calls = []
    orig = gemm._TiedDecoder.backward

    def spy(ctx, dy):
        calls.append(dy.stride(0))
        return orig(ctx, dy)
    gemm._TiedDecoder.backward = staticmethod(spy)
    try:
        w, b = wv.read(torch.bfloat16), bv.read(torch.bfloat16)
        logits = ops.tied_decoder(h, w, b)
        assert logits.shape == (M, Vn) and logits.stride(0) == 30720
        loss = kernels.softmax_xent(logits, labels).mean()
        loss.backward()
    finally:
        gemm._TiedDecoder.backward = orig
    assert calls == [30720], "the padded decoder backward did not run on the zero-padded logit gradient"
    hf = h.detach().float().requires_grad_(True)
    wf = wv.shadow.float().requires_grad_(True)
    bf = bv.shadow.float().requires_grad_(True)
    lf = hf @ wf.t() + bf
    assert _rel(logits.float(), lf) < 1e-2
    torch.nn.functional.cross_entropy(lf, labels).backward()
    assert _rel(h.grad, hf.grad) < 1e-2
    assert _rel(wv.grad, wf.grad) < 2e-2
    assert _rel(bv.grad, bf.grad) < 1e-2
    assert not wv.grad_padded[Vn:].any() and not bv.grad_padded[Vn:].any()


def test_bn_backward_finalize_on_wgrad_launch_matches_inline(monkeypatch):
    """The BN backward finalize run by extra workgroups of the conv's weight-gradient launch (MDTF_BN_WG_FIN, the
    default: csrc/conv_igemm.hip fin_bwd_block) == the finalize launch inside the BN backward: same loss and the
    same gradients on a two-stage ResNet (up to the order of fp32 atomics); the fused path must actually run."""
    from mdtf.ops import bn
    torch.manual_seed(10)
    x = torch.randn(8, 64, 64, 3)
    y = torch.randint(0, 16, (8,))
    monkeypatch.setattr(bn, "EARLY_FIN", False)
    monkeypatch.setattr(bn, "WG_FIN", True)
    n0 = bn.WG_FIN_USED[0]
    lf, gf = _one_step(DEV, torch.bfloat16, x, y, blocks=[1, 1], grads=True)
    assert bn.WG_FIN_USED[0] > n0
    monkeypatch.setattr(bn, "WG_FIN", False)
    n1 = bn.WG_FIN_USED[0]
    li, gi = _one_step(DEV, torch.bfloat16, x, y, blocks=[1, 1], grads=True)
    assert bn.WG_FIN_USED[0] == n1
    assert lf == li
    for k in gi:
        assert _rel(gf[k], gi[k]) < 1e-4, (k, _rel(gf[k], gi[k]))


def test_bn_backward_early_finalize_matches_inline(monkeypatch):
    """The BN backward finalize issued early on a side stream (MDTF_BN_EARLY_FIN=1: right after the data gradient
    that completes its statistics, beside the conv weight gradient) == the finalize inside the BN backward:
    same loss and the same gradients on a two-stage ResNet (up to the order of the fp32 weight-gradient atomics,
    which differs run to run); the early path must actually run."""
    from mdtf.ops import bn
    torch.manual_seed(9)
    x = torch.randn(8, 64, 64, 3)
    y = torch.randint(0, 16, (8,))
    monkeypatch.setattr(bn, "WG_FIN", False)          # inline = the finalize launch inside the BN backward
    monkeypatch.setattr(bn, "EARLY_FIN", True)
    n0 = bn.EARLY_USED[0]
    le, ge = _one_step(DEV, torch.bfloat16, x, y, blocks=[1, 1], grads=True)
    assert bn.EARLY_USED[0] > n0
    monkeypatch.setattr(bn, "EARLY_FIN", False)
    n1 = bn.EARLY_USED[0]
    li, gi = _one_step(DEV, torch.bfloat16, x, y, blocks=[1, 1], grads=True)
    assert bn.EARLY_USED[0] == n1
    assert le == li
    for k in gi:
        assert _rel(ge[k], gi[k]) < 1e-4, (k, _rel(ge[k], gi[k]))


def test_bn_on_consumer_conv_matches_separate_apply(monkeypatch):
    """A BN + ReLU applied by the 1x1 conv consuming it (MDTF_BN_ON_CONSUMER: finalize only, the weight-stationary
    kernel's operand loads apply scale / shift / ReLU and write the BN output, csrc/conv_ws.hip
    mdtf_conv_ws_bna) == the separate apply pass: the BN output and the conv + BN output up to the order of the
    statistics atomics, and the BN output against an fp32 PyTorch reference; stage-1 and stage-2 conv3 shapes."""
    from mdtf.ops import bn
    torch.manual_seed(11)
    for hw, c in ((56, 64), (28, 128)):
        x = torch.randn(2, hw, hw, c, device=DEV).bfloat16()
        w2 = (torch.randn(3, 3, c, c, device=DEV) * (1.0 / (3 * c ** 0.5))).bfloat16()
        w3 = (torch.randn(1, 1, c, 4 * c, device=DEV) * (1.0 / c ** 0.5)).bfloat16()
        g = torch.rand(c, device=DEV) + 0.5
        b = torch.randn(c, device=DEV) * 0.2
        g3, b3 = torch.ones(4 * c, device=DEV), torch.zeros(4 * c, device=DEV)

        def run(on):
            monkeypatch.setattr(bn, "ON_CONSUMER", on)
            n0 = bn.ON_CONSUMER_USED[0]
            a = ops.conv_bn(x, w2, g, b, torch.zeros(c, device=DEV), torch.ones(c, device=DEV), 1, "SAME", True, 0.9,
                            1e-5, True, None, on_consumer=True)
            z = ops.conv_bn(a, w3, g3, b3, torch.zeros(4 * c, device=DEV), torch.ones(4 * c, device=DEV), 1, "SAME",
                            True, 0.9, 1e-5, False, None)
            torch.cuda.synchronize()
            return a.float().clone(), z.float().clone(), bn.ON_CONSUMER_USED[0] - n0

        a1, z1, used1 = run(True)
        a0, z0, used0 = run(False)
        assert used1 == 1 and used0 == 0, (hw, used1, used0)
        # (not bitwise: the conv2 statistics are fp32 atomics, their order -- and the last bit of scale / shift --
        # differs run to run)
        assert _rel(a1, a0) < 1e-4, (hw, _rel(a1, a0))
        assert _rel(z1, z0) < 1e-3, (hw, _rel(z1, z0))
        # fp32 reference of the pair
        xf = x.float().permute(0, 3, 1, 2)
        h = torch.nn.functional.conv2d(xf, w2.float().permute(3, 2, 0, 1), padding=1)
        mu, var = h.mean((0, 2, 3), keepdim=True), h.var((0, 2, 3), unbiased=False, keepdim=True)
        ar = torch.relu((h - mu) / torch.sqrt(var + 1e-5) * g.view(1, -1, 1, 1) + b.view(1, -1, 1, 1))
        assert _rel(a1, ar.permute(0, 2, 3, 1)) < 2e-2, (hw, _rel(a1, ar.permute(0, 2, 3, 1)))


def test_bn_on_consumer_resnet_step_matches(monkeypatch):
    """A two-stage ResNet step at 224 x 224 (stage-1 / stage-2 conv3 on the weight-stationary kernel) with the
    conv2 BN + ReLU applied by conv3 == the separate apply pass: the loss and every gradient (the backward reads
    the BN output and ReLU mask the fused kernel wrote)."""
    from mdtf.ops import bn
    torch.manual_seed(12)
    x = torch.randn(2, 224, 224, 3)
    y = torch.randint(0, 16, (2,))
    monkeypatch.setattr(bn, "ON_CONSUMER", True)
    n0 = bn.ON_CONSUMER_USED[0]
    l1, g1 = _one_step(DEV, torch.bfloat16, x, y, blocks=[1, 1], grads=True)
    assert bn.ON_CONSUMER_USED[0] - n0 >= 2                # stage-1 and stage-2 conv3 (per forward the step runs)
    monkeypatch.setattr(bn, "ON_CONSUMER", False)
    l0, g0 = _one_step(DEV, torch.bfloat16, x, y, blocks=[1, 1], grads=True)
    _, g0b = _one_step(DEV, torch.bfloat16, x, y, blocks=[1, 1], grads=True)     # the run-to-run noise floor
    assert abs(l1 - l0) <= 1e-3 * abs(l0), (l1, l0)
    errs = {k: (_rel(g1[k], g0[k]), _rel(g0b[k], g0[k])) for k in g0}
    bad = {k: e for k, e in errs.items() if e[0] > max(1e-3, 4 * e[1])}
    assert not bad, bad
