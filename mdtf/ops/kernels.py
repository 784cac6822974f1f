"""Autograd wrappers of the memory-bound HIP kernels in ``csrc/kernels.hip``."""
import torch

from . import _native as N
from ..train import variables as V

N.register("mdtf_bias_act_fwd", [N.P, N.P, N.P, N.P, N.L, N.I, N.I, N.P])
N.register("mdtf_act_bwd", [N.P, N.P, N.P, N.P, N.L, N.I, N.P])
N.register("mdtf_colsum", [N.P, N.L, N.I, N.P, N.P, N.P])
N.register("mdtf_mask_mul", [N.P, N.P, N.P, N.L, N.I, N.P])
N.register("mdtf_colsum_ws", [N.L, N.I], restype=N.L)
N.register("mdtf_pool_fwd", [N.I, N.P, N.P, N.P] + [N.I] * 12 + [N.P])
N.register("mdtf_pool_bwd", [N.I, N.P, N.P, N.P] + [N.I] * 12 + [N.P])
N.register("mdtf_gap_fwd", [N.P, N.P, N.I, N.I, N.I, N.P])
N.register("mdtf_gap_bwd", [N.P, N.P, N.I, N.I, N.I, N.P])
N.register("mdtf_xent_fwd", [N.P, N.I, N.P, N.I, N.I, N.L, N.P, N.P, N.P])
N.register("mdtf_xent_bwd", [N.P, N.I, N.P, N.P, N.P, N.P, N.I, N.I, N.L, N.L, N.P])
N.register("mdtf_transpose_brs", [N.P, N.P, N.I, N.I, N.I, N.I, N.P])
N.register("mdtf_lrn_fwd", [N.P, N.P, N.P, N.L, N.I, N.I, N.F, N.F, N.F, N.P])
N.register("mdtf_lrn_bwd", [N.P, N.P, N.P, N.P, N.P, N.L, N.I, N.I, N.F, N.F, N.P])

_ACT = {None: 0, "relu": 1, "gelu": 2}


def _bf16(x, what):
    if x.dtype != torch.bfloat16:
        raise TypeError("mdtf %s kernel expects bf16, got %s" % (what, x.dtype))
    return x.contiguous()


def colsum_into(x2d, out):
    """``out += x2d.sum(0)`` for a bf16 [M, C] matrix and an fp32 [C] ``out``."""
    M, C = x2d.shape
    ws = torch.empty(max(N.fn("mdtf_colsum_ws")(M, C), 1), dtype=torch.float32, device=x2d.device)
    N.check(N.fn("mdtf_colsum")(N.ptr(x2d), M, C, N.ptr(out), N.ptr(ws), N.stream_ptr()), "colsum")
    return out


def colsum(x2d):
    """Column sums of a bf16 [M, C] matrix -> fp32 [C]."""
    return colsum_into(x2d, torch.zeros(x2d.shape[1], dtype=torch.float32, device=x2d.device))


class _BiasAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, bias, act):
        x = _bf16(x, "bias_act")
        C = x.shape[-1]
        M = x.numel() // C
        y = torch.empty_like(x)
        pre = torch.empty_like(x) if act == 2 else None
        b = bias.detach().float().contiguous() if bias is not None else None
        N.check(N.fn("mdtf_bias_act_fwd")(N.ptr(x), N.ptr(b), N.ptr(y), N.ptr(pre), M, C, act, N.stream_ptr()),
                "bias_act")
        ctx.act = act
        ctx.has_bias = bias is not None
        ctx.bias_dtype = bias.dtype if bias is not None else None
        ctx.sink = V.grad_sink(bias) if bias is not None else None
        ctx.bias = bias
        ctx.save_for_backward(y if act == 1 else pre)
        return y

    @staticmethod
    def backward(ctx, dy):
        (saved,) = ctx.saved_tensors
        dy = dy.contiguous()
        if ctx.act == 0:
            dx = dy
        else:
            dx = torch.empty_like(dy)
            pre = saved if ctx.act == 2 else None
            y = saved if ctx.act == 1 else None
            N.check(N.fn("mdtf_act_bwd")(N.ptr(dy), N.ptr(pre), N.ptr(y), N.ptr(dx), dy.numel(), ctx.act,
                                         N.stream_ptr()), "act_bwd")
        db = None
        if ctx.has_bias:
            C = dx.shape[-1]
            if ctx.sink is not None:       # column sums accumulate straight into the fp32 grad slot
                colsum_into(dx.view(-1, C), ctx.sink.grad)
                db = V.grad_marker(ctx.bias)
            else:
                db = colsum(dx.reshape(-1, C)).to(ctx.bias_dtype)
        return dx, db, None


def bias_act(x, b, act="relu"):
    return _BiasAct.apply(x, b, _ACT[act])


def relu(x):
    return _BiasAct.apply(x, None, 1)


# ---------------------------------------------------------------- pooling
class _Pool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, is_max, k, s, pads, out_hw):
        x = _bf16(x, "pool")
        n, h, w, c = x.shape
        oh, ow = out_hw
        y = torch.empty((n, oh, ow, c), dtype=x.dtype, device=x.device)
        arg = torch.empty((n, oh, ow, c), dtype=torch.uint8, device=x.device) if is_max else None
        geo = [n, h, w, c, oh, ow, k[0], k[1], s[0], s[1], pads[0], pads[2]]
        N.check(N.fn("mdtf_pool_fwd")(int(is_max), N.ptr(x), N.ptr(y), N.ptr(arg), *geo, N.stream_ptr()), "pool_fwd")
        ctx.geo = geo
        ctx.is_max = is_max
        if is_max:
            ctx.save_for_backward(arg)
        # fanned-out output (a ResNet stem pool feeds conv1 AND the projection shortcut): the
        # consumers' dgrads accumulate in place instead of autograd adding their gradients
        from . import actsink
        ctx.set_materialize_grads(False)
        ctx.out_sink = actsink.attach(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        if ctx.out_sink is not None:
            dy = ctx.out_sink.take(dy)
        if dy is None:
            return None, None, None, None, None, None
        dy = dy.contiguous()
        geo = ctx.geo
        arg = ctx.saved_tensors[0] if ctx.is_max else None
        dx = torch.empty((geo[0], geo[1], geo[2], geo[3]), dtype=dy.dtype, device=dy.device)
        N.check(N.fn("mdtf_pool_bwd")(int(ctx.is_max), N.ptr(dy), N.ptr(arg), N.ptr(dx), *geo, N.stream_ptr()),
                "pool_bwd")
        return dx, None, None, None, None, None


def max_pool(x, k, s, pads, out_hw):
    return _Pool.apply(x, True, k, s, pads, out_hw)


def avg_pool(x, k, s, pads, out_hw):
    return _Pool.apply(x, False, k, s, pads, out_hw)


class _GAP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = _bf16(x, "global_avg_pool")
        n, h, w, c = x.shape
        y = torch.empty((n, c), dtype=x.dtype, device=x.device)
        N.check(N.fn("mdtf_gap_fwd")(N.ptr(x), N.ptr(y), n, h * w, c, N.stream_ptr()), "gap_fwd")
        ctx.shape = (n, h, w, c)
        return y

    @staticmethod
    def backward(ctx, dy):
        n, h, w, c = ctx.shape
        dy = dy.contiguous()
        dx = torch.empty((n, h, w, c), dtype=dy.dtype, device=dy.device)
        N.check(N.fn("mdtf_gap_bwd")(N.ptr(dy), N.ptr(dx), n, h * w, c, N.stream_ptr()), "gap_bwd")
        return dx


def global_avg_pool(x):
    return _GAP.apply(x)


# ---------------------------------------------------------------- softmax xent
class _Xent(torch.autograd.Function):
    """Rows may be strided (``logits.stride(0) >= K``, unit column stride): the padded MLM decoder hands over a
    [rows, 30522] view of its [rows, 30720] logits.  The gradient then comes back as the same view of a zero-padded
    [rows, 30720] buffer, which the decoder's backward reads whole (``gemm.tied_decoder``)."""

    @staticmethod
    def forward(ctx, logits, labels):
        if logits.dtype not in (torch.bfloat16, torch.float32):
            logits = logits.float()
        if logits.stride(1) != 1 or logits.stride(0) < logits.shape[1]:
            logits = logits.contiguous()
        labels = labels.to(torch.int64).contiguous()
        n, k = logits.shape
        loss = torch.empty(n, dtype=torch.float32, device=logits.device)
        lse = torch.empty_like(loss)
        is_bf = int(logits.dtype == torch.bfloat16)
        N.check(N.fn("mdtf_xent_fwd")(N.ptr(logits), is_bf, N.ptr(labels), n, k, logits.stride(0), N.ptr(loss),
                                      N.ptr(lse), N.stream_ptr()), "xent_fwd")
        ctx.save_for_backward(logits, labels, lse)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        logits, labels, lse = ctx.saved_tensors
        n, k = logits.shape
        ldi = logits.stride(0)
        ldo = ldi if (ldi != k and ldi % 8 == 0 and logits.dtype == torch.bfloat16) else k
        dl = torch.empty((n, ldo), dtype=logits.dtype, device=logits.device)
        dloss = dloss.float().contiguous()
        N.check(N.fn("mdtf_xent_bwd")(N.ptr(logits), int(logits.dtype == torch.bfloat16), N.ptr(labels), N.ptr(lse),
                                      N.ptr(dloss), N.ptr(dl), n, k, ldi, ldo, N.stream_ptr()), "xent_bwd")
        if ldo == k:
            return dl, None
        if logits.data_ptr() % 16 or dl.data_ptr() % 16:
            # mdtf_xent_bwd zero-fills the pad columns only on its 16-B vector path (kernels.hip:863-870); the
            # generic kernel leaves them as torch.empty made them, and the tied decoder reads whole rows
            dl[:, k:].zero_()
        from . import gemm
        if len(gemm._PADDED_GRADS) > 16:
            gemm._PADDED_GRADS.clear()
        gemm._PADDED_GRADS[dl.data_ptr()] = ldo     # zero-padded: the tied decoder may read the whole rows
        return dl[:, :k], None


def softmax_xent(logits, labels):
    return _Xent.apply(logits, labels)


# ---------------------------------------------------------------- layout
def transpose_brs(x, B, R, S):
    """[B, R, S] -> [B, S, R] for 2- or 4-byte dtypes."""
    x = x.contiguous()
    out = torch.empty((B, S, R), dtype=x.dtype, device=x.device)
    N.check(N.fn("mdtf_transpose_brs")(N.ptr(x), N.ptr(out), B, R, S, x.element_size(), N.stream_ptr()),
            "transpose")
    return out


class _Layout(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, to_nhwc):
        ctx.to_nhwc = to_nhwc
        if to_nhwc:
            n, c, h, w = x.shape
            return transpose_brs(x, n, c, h * w).view(n, h, w, c)
        n, h, w, c = x.shape
        return transpose_brs(x, n, h * w, c).view(n, c, h, w)

    @staticmethod
    def backward(ctx, g):
        return _Layout.apply(g, not ctx.to_nhwc), None


def nchw_to_nhwc(x):
    return _Layout.apply(x, True)


def nhwc_to_nchw(x):
    return _Layout.apply(x, False)


# ---------------------------------------------------------------- LRN
class _LRN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, r, bias, alpha, beta):
        x = _bf16(x, "lrn")
        c = x.shape[-1]
        p = x.numel() // c
        y = torch.empty_like(x)
        d = torch.empty(x.shape, dtype=torch.float32, device=x.device)
        N.check(N.fn("mdtf_lrn_fwd")(N.ptr(x), N.ptr(y), N.ptr(d), p, c, r, bias, alpha, beta, N.stream_ptr()),
                "lrn_fwd")
        ctx.save_for_backward(x, y, d)
        ctx.args = (r, alpha, beta)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, y, d = ctx.saved_tensors
        r, alpha, beta = ctx.args
        dy = dy.contiguous()
        dx = torch.empty_like(x)
        c = x.shape[-1]
        N.check(N.fn("mdtf_lrn_bwd")(N.ptr(dy), N.ptr(x), N.ptr(y), N.ptr(d), N.ptr(dx), x.numel() // c, c, r, alpha,
                                     beta, N.stream_ptr()), "lrn_bwd")
        return dx, None, None, None, None


def lrn(x, depth_radius, bias, alpha, beta):
    return _LRN.apply(x, int(depth_radius), float(bias), float(alpha), float(beta))

