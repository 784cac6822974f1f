"""Neural-network ops on NHWC tensors (TF conventions), dispatching to HIP kernels.

Every op here has two implementations:

* a HIP/CDNA4 kernel in ``mdtf/csrc`` used for GPU tensors (``mdtf.ops._native``);
* a plain PyTorch implementation used for CPU tensors (unit tests, the LeNet
  CPU config) and, with ``MDTF_KERNELS=torch``, as the stock-PyTorch
  comparator on the GPU.

Reference call sites: ``distribute_tools.py:76-207`` (conv2d, bias_add, relu,
conv2d_transpose, max/avg pool, moments/batch_normalization, lrn, matmul).
Layouts follow TF: activations NHWC, conv filters HWIO (``[kh, kw, cin, cout]``),
transposed-conv filters ``[kh, kw, cout, cin]``, FC weights ``[in, out]``.
"""
import torch
import torch.nn.functional as F

from . import _native
from .padding import conv_geometry, pair

# ---------------------------------------------------------------------------
# elementwise
# ---------------------------------------------------------------------------


def relu(x):
    if _native.use_native(x):
        from . import kernels
        return kernels.relu(x)
    return torch.relu(x)


def bias_add(x, b):
    """Per-channel bias on the last (C) dim (``tf.nn.bias_add``, NHWC)."""
    return x + b.to(x.dtype)


def bias_add_relu(x, b):
    if _native.use_native(x):
        from . import kernels
        return kernels.bias_act(x, b, act="relu")
    return torch.relu(x + b.to(x.dtype))


# ---------------------------------------------------------------------------
# convolution
# ---------------------------------------------------------------------------


def _torch_conv_nhwc(x, w_hwio, sh, sw, pads, dh, dw, groups=1):
    pt, pb, pl, pr = pads
    xc = x.permute(0, 3, 1, 2)                   # NCHW view, channels_last strides
    if not (pt == pb and pl == pr):
        xc = F.pad(xc, (pl, pr, pt, pb))
        ph, pw = 0, 0
    else:
        ph, pw = pt, pl
    wt = w_hwio.permute(3, 2, 0, 1)              # OIHW view
    if x.is_cuda:
        wt = wt.contiguous(memory_format=torch.channels_last)
    y = F.conv2d(xc, wt.to(x.dtype), None, (sh, sw), (ph, pw), (dh, dw), groups)
    return y.permute(0, 2, 3, 1)


def conv2d(x, w, strides=1, padding="SAME", dilations=1, bias=None, act=None, name=None):
    """2-D convolution, NHWC input, HWIO filter (``tf.nn.conv2d``).

    ``strides``/``dilations`` accept an int, ``[sh, sw]`` or TF's ``[1, sh, sw, 1]``.
    ``padding`` is 'SAME', 'VALID', an int, ``(ph, pw)`` or ``(pt, pb, pl, pr)``.
    Optional fused epilogue: ``bias`` (per output channel) and ``act='relu'``.
    """
    n, h, wd, c = x.shape
    kh, kw, ci, co = w.shape
    if ci != c:
        raise ValueError("conv2d: input has %d channels, filter expects %d" % (c, ci))
    sh, sw = pair(strides)
    dh, dw = pair(dilations)
    oh, ow, pt, pb, pl, pr = conv_geometry(h, wd, kh, kw, (sh, sw), padding, (dh, dw))
    if _native.use_native(x):
        from . import conv as conv_mod
        return conv_mod.conv2d_nhwc(x, w, (sh, sw), (pt, pb, pl, pr), (dh, dw), bias=bias, act=act)
    y = _torch_conv_nhwc(x, w, sh, sw, (pt, pb, pl, pr), dh, dw)
    if bias is not None:
        y = y + bias.to(y.dtype)
    if act == "relu":
        y = torch.relu(y)
    return y


def conv2d_transpose(x, w, output_shape, strides=1, padding="SAME", name=None):
    """Transposed conv (``tf.nn.conv2d_transpose``): filter ``[kh, kw, cout, cin]``.

    Implemented as the data-gradient of ``conv2d`` (the same math the GPU
    kernel uses: conv dgrad reused as a forward).
    """
    n, oh, ow, co = [int(s) for s in output_shape]
    kh, kw, wco, wci = w.shape
    if wci != x.shape[-1] or wco != co:
        raise ValueError("conv2d_transpose: filter %s incompatible with input %s / output %s" % (
            tuple(w.shape), tuple(x.shape), tuple(output_shape)))
    sh, sw = pair(strides)
    gh, gw, pt, pb, pl, pr = conv_geometry(oh, ow, kh, kw, (sh, sw), padding)
    if (gh, gw) != tuple(x.shape[1:3]):
        raise ValueError("conv2d_transpose: output_shape %s inconsistent with input %s" % (
            tuple(output_shape), tuple(x.shape)))
    if _native.use_native(x):
        from . import conv as conv_mod
        return conv_mod.conv2d_dgrad_nhwc(x, w, (n, oh, ow, co), (sh, sw), (pt, pb, pl, pr))
    xc = x.permute(0, 3, 1, 2)
    wt = w.permute(3, 2, 0, 1).to(x.dtype)       # [cin(x), cout, kh, kw] == conv_transpose weight layout
    # conv_transpose2d with asymmetric pads: compute full then crop.
    y = F.conv_transpose2d(xc, wt, None, (sh, sw), 0)
    y = y[:, :, pt:pt + oh, pl:pl + ow]
    if y.shape[2] < oh or y.shape[3] < ow:
        y = F.pad(y, (0, ow - y.shape[3], 0, oh - y.shape[2]))
    return y.permute(0, 2, 3, 1)


# ---------------------------------------------------------------------------
# pooling
# ---------------------------------------------------------------------------


def _pool_args(ksize, strides):
    return pair(ksize), pair(strides)


def max_pool(x, ksize=(1, 2, 2, 1), strides=(1, 2, 2, 1), padding="SAME", name=None):
    (kh, kw), (sh, sw) = _pool_args(ksize, strides)
    n, h, w, c = x.shape
    oh, ow, pt, pb, pl, pr = conv_geometry(h, w, kh, kw, (sh, sw), padding)
    if _native.use_native(x):
        from . import kernels
        return kernels.max_pool(x, (kh, kw), (sh, sw), (pt, pb, pl, pr), (oh, ow))
    xc = x.permute(0, 3, 1, 2)
    if pt or pb or pl or pr:
        xc = F.pad(xc, (pl, pr, pt, pb), value=float("-inf"))
    y = F.max_pool2d(xc, (kh, kw), (sh, sw))
    return y.permute(0, 2, 3, 1)[:, :oh, :ow, :]


def avg_pool(x, ksize=(1, 2, 2, 1), strides=(1, 2, 2, 1), padding="SAME", name=None):
    """Average pool; SAME padding averages over valid elements only (TF semantics)."""
    (kh, kw), (sh, sw) = _pool_args(ksize, strides)
    n, h, w, c = x.shape
    oh, ow, pt, pb, pl, pr = conv_geometry(h, w, kh, kw, (sh, sw), padding)
    if _native.use_native(x):
        from . import kernels
        return kernels.avg_pool(x, (kh, kw), (sh, sw), (pt, pb, pl, pr), (oh, ow))
    xc = x.permute(0, 3, 1, 2)
    ones = torch.ones((1, 1, h, w), dtype=x.dtype, device=x.device)
    if pt or pb or pl or pr:
        xc = F.pad(xc, (pl, pr, pt, pb))
        ones = F.pad(ones, (pl, pr, pt, pb))
    s = F.avg_pool2d(xc, (kh, kw), (sh, sw)) * (kh * kw)
    cnt = F.avg_pool2d(ones, (kh, kw), (sh, sw)) * (kh * kw)
    y = s / cnt
    return y.permute(0, 2, 3, 1)[:, :oh, :ow, :]


def global_avg_pool(x):
    """Mean over H, W of an NHWC tensor -> [N, C] (fp32 accumulation)."""
    if _native.use_native(x):
        from . import kernels
        return kernels.global_avg_pool(x)
    return x.float().mean(dim=(1, 2)).to(x.dtype)


# ---------------------------------------------------------------------------
# normalisation
# ---------------------------------------------------------------------------


def moments(x, axes, keep_dims=False):
    """``tf.nn.moments``: (mean, biased variance) over ``axes``."""
    xf = x.float()
    mean = xf.mean(dim=tuple(axes), keepdim=True)
    var = ((xf - mean) ** 2).mean(dim=tuple(axes), keepdim=True)
    if not keep_dims:
        mean = mean.squeeze(tuple(axes)) if len(axes) else mean
        var = var.squeeze(tuple(axes)) if len(axes) else var
    return mean, var


def batch_normalization(x, mean, variance, offset, scale, variance_epsilon):
    """``tf.nn.batch_normalization`` with broadcasting statistics."""
    inv = torch.rsqrt(variance + variance_epsilon)
    if scale is not None:
        inv = inv * scale
    y = (x.float() - mean) * inv
    if offset is not None:
        y = y + offset
    return y.to(x.dtype)


def batch_norm(x, gamma, beta, moving_mean, moving_var, training=True, decay=0.9, epsilon=1e-3,
               relu=False, residual=None):
    """Fused per-channel batch norm over N·H·W of an NHWC tensor.

    Training: batch statistics (fp32 Welford/sum-of-squares), moving averages
    updated in place (``moving = decay*moving + (1-decay)*batch``, unbiased
    variance), optional fused residual add and ReLU:
    ``y = relu(gamma * (x - mean) * rsqrt(var + eps) + beta [+ residual])``.
    """
    if _native.use_native(x):
        from . import bn
        return bn.batch_norm_nhwc(x, gamma, beta, moving_mean, moving_var, training, decay, epsilon,
                                  relu, residual)
    c = x.shape[-1]
    x2 = x.reshape(-1, c)
    if training:
        xf = x2.float()
        mean = xf.mean(0)
        var = xf.var(0, unbiased=False)
        with torch.no_grad():
            if moving_mean is not None:
                m = x2.shape[0]
                moving_mean.mul_(decay).add_(mean.detach(), alpha=1 - decay)
                moving_var.mul_(decay).add_(var.detach() * (m / max(m - 1, 1)), alpha=1 - decay)
    else:
        mean, var = moving_mean.float(), moving_var.float()
    inv = torch.rsqrt(var + epsilon)
    g = gamma.float() if gamma is not None else 1.0
    b = beta.float() if beta is not None else 0.0
    y = (x2.float() - mean) * (inv * g) + b
    y = y.reshape(x.shape)
    if residual is not None:
        y = y + residual.float()
    if relu:
        y = torch.relu(y)
    return y.to(x.dtype)


def conv_bn(x, w, gamma, beta, moving_mean, moving_var, strides=1, padding="SAME", training=True, decay=0.9,
            epsilon=1e-5, relu=True, residual=None, defer=False, pool=None, on_consumer=False):
    """conv2d (no bias) -> batch_norm (+residual) (+ReLU).

    On the GPU the conv epilogue emits the per-channel Σy/Σy² partials, so the
    BN statistics pass over y disappears (BN runs finalize + apply only).
    ``defer`` (no ReLU / residual; a projection shortcut): on the GPU return a :class:`bn.DeferredBN` that
    the residual BN consuming it applies in its own pass; elsewhere the normalised tensor as usual.
    ``pool = (ksize, stride, padding)``: a max pool follows (the ResNet stem); on the GPU BN + ReLU + pool run
    as one pass (``bn.bn_relu_maxpool_nhwc``).
    ``on_consumer``: the output feeds only a 1x1 conv that may apply the BN + ReLU to its operand on the GPU
    (``bn.ON_CONSUMER``).
    """
    n, h, wd, c = x.shape
    kh, kw, ci, co = w.shape
    sh, sw = pair(strides)
    oh, ow, pt, pb, pl, pr = conv_geometry(h, wd, kh, kw, (sh, sw), padding)
    if _native.use_native(x) and training:
        from . import conv as conv_mod
        from . import bn
        defer = defer and not relu and residual is None and bn.DEFER_SHORTCUT
        y, stats = conv_mod.conv2d_stats_nhwc(x, w, (sh, sw), (pt, pb, pl, pr), (1, 1), private=defer)
        if defer and stats is not None:
            return bn.DeferredBN(y, gamma, beta, moving_mean, moving_var, decay, epsilon, stats)
        if pool is not None and relu and residual is None and stats is not None and bn.FUSED_STEM:
            (pkh, pkw), (psh, psw) = _pool_args(pool[0], pool[1])
            poh, pow_, ppt, _, ppl, _ = conv_geometry(oh, ow, pkh, pkw, (psh, psw), pool[2])
            return bn.bn_relu_maxpool_nhwc(y, gamma, beta, moving_mean, moving_var, decay, epsilon, stats,
                                           (poh, pow_, pkh, pkw, psh, psw, ppt, ppl))
        y = bn.batch_norm_nhwc(y, gamma, beta, moving_mean, moving_var, True, decay, epsilon, relu, residual,
                               stats=stats, on_consumer=on_consumer and pool is None)
        return y if pool is None else max_pool(y, pool[0], pool[1], pool[2])
    y = conv2d(x, w, strides, (pt, pb, pl, pr))
    y = batch_norm(y, gamma, beta, moving_mean, moving_var, training, decay, epsilon, relu, residual)
    return y if pool is None else max_pool(y, pool[0], pool[1], pool[2])


def local_response_normalization(x, depth_radius=5, bias=1.0, alpha=1.0, beta=0.5, name=None):
    """``tf.nn.lrn`` over the channel (last) axis of an NHWC tensor."""
    if _native.use_native(x):
        from . import kernels
        return kernels.lrn(x, depth_radius, bias, alpha, beta)
    xf = x.float()
    sq = (xf * xf).permute(0, 3, 1, 2)           # N C H W
    # sum over window [c - r, c + r]
    sq = F.pad(sq.unsqueeze(1), (0, 0, 0, 0, depth_radius, depth_radius)).squeeze(1)
    win = sq.unfold(1, 2 * depth_radius + 1, 1).sum(-1)
    y = xf / (bias + alpha * win.permute(0, 2, 3, 1)) ** beta
    return y.to(x.dtype)


lrn = local_response_normalization


def layer_norm(x, gamma, beta, epsilon=1e-12, residual=None):
    """LayerNorm over the last axis (optionally of ``x + residual``, fused on the GPU)."""
    from . import transformer
    return transformer.layer_norm(x, gamma, beta, epsilon, residual)


# ---------------------------------------------------------------------------
# dense
# ---------------------------------------------------------------------------


def matmul(a, b, transpose_a=False, transpose_b=False):
    if transpose_a:
        a = a.transpose(-1, -2)
    if transpose_b:
        b = b.transpose(-1, -2)
    if _native.use_native(a) and a.dim() == 2 and b.dim() == 2:
        from . import gemm
        return gemm.matmul(a, b.to(a.dtype))
    return torch.matmul(a, b.to(a.dtype))


def dense(x, w, b=None, act=None):
    """``x @ w + b`` with optional fused activation ('relu' | 'gelu' | None)."""
    if _native.use_native(x):
        from . import gemm
        return gemm.dense(x, w, b, act)
    y = torch.matmul(x, w.to(x.dtype))
    if b is not None:
        y = y + b.to(y.dtype)
    if act == "relu":
        y = torch.relu(y)
    elif act == "gelu":
        y = F.gelu(y.float(), approximate="tanh").to(y.dtype)
    return y


def ffn(x, w1, b1, w2, b2, act="gelu"):
    """``act(x @ w1 + b1) @ w2 + b2``: a feed-forward block (native: the activation backward is fused into the
    second layer's data gradient)."""
    if _native.use_native(x):
        from . import gemm
        return gemm.ffn(x, w1, b1, w2, b2, act)
    return dense(dense(x, w1, b1, act), w2, b2)


def dense_multi(x, ws, bs, act=None):
    """One GEMM for several ``[K, N_i]`` weights sharing input ``x``; outputs concatenated on the last axis."""
    if _native.use_native(x):
        from . import gemm
        return gemm.dense_multi(x, ws, bs, act)
    w = torch.cat([t.to(x.dtype) for t in ws], 1)
    b = torch.cat(list(bs), 0) if bs[0] is not None else None
    return dense(x, w, b, act)


def dense_transposed(x, w, b=None):
    """``x @ w^T + b`` for w [N, K] (tied embedding decoders)."""
    if _native.use_native(x):
        from . import gemm
        return gemm.dense_transposed(x, w, b)
    y = torch.matmul(x, w.to(x.dtype).t())
    return y + b.to(y.dtype) if b is not None else y


def tied_decoder(x, w, b):
    """``x @ w^T + b`` of a decoder tied to an embedding variable: on the GPU over the vocabulary padded to the
    variables' ``pad_rows`` (``gemm.tied_decoder``), else :func:`dense_transposed`."""
    if _native.use_native(x):
        from . import gemm
        return gemm.tied_decoder(x, w, b)
    return dense_transposed(x, w, b)


def decoder_pad_rows(vocab):
    """Zero rows a tied embedding reserves for :func:`tied_decoder` (0 when the padded path is off)."""
    from . import gemm
    return gemm.decoder_pad_rows(vocab) if gemm.DEC_SPLIT > 0 else 0


def gelu(x):
    return F.gelu(x.float(), approximate="tanh").to(x.dtype)


def dropout(x, rate, training=True):
    if not training or rate <= 0:
        return x
    return F.dropout(x, rate, True)


# ---------------------------------------------------------------------------
# losses
# ---------------------------------------------------------------------------


def sparse_softmax_cross_entropy_with_logits(labels, logits):
    """Per-example cross entropy with integer labels (fp32 math)."""
    if _native.use_native(logits) and logits.dim() == 2:
        from . import kernels
        return kernels.softmax_xent(logits, labels)
    return F.cross_entropy(logits.float(), labels.long(), reduction="none")


def softmax_cross_entropy_with_logits(labels, logits):
    lf = logits.float()
    return -(labels.float() * torch.log_softmax(lf, dim=-1)).sum(-1)


def l2_loss(t):
    """``sum(t ** 2) / 2`` in fp32 (``tf.nn.l2_loss``)."""
    tf_ = t.float()
    return (tf_ * tf_).sum() * 0.5


def mean_squared_error(labels, predictions):
    return ((predictions.float() - labels.float()) ** 2).mean()


def reduce_mean(t, axis=None):
    t = t if not isinstance(t, (list, tuple)) else torch.stack([torch.as_tensor(x).float() for x in t])
    return t.float().mean() if axis is None else t.float().mean(dim=axis)


def add_n(ts):
    out = ts[0]
    for t in ts[1:]:
        out = out + t
    return out
