"""Fused optimizer updates over flat parameter buffers.

One launch updates a whole parameter group in place: fp32 master, optimizer
state, and the bf16 compute shadow (so the next forward needs no cast
kernels), with the data-parallel ``1/N`` gradient scale and L2 weight decay
folded in.  Reference: the optimizer is ``tf.train.AdamOptimizer(0.001)``
(``distribute.py:26``) applied per variable on PS CPUs
(``distribute_train.py:151-158``); SURVEY §2.5 K9 (l2_loss×wd) and K13
(fused multi-tensor Adam/SGD).

GPU tensors run ``mdtf_fused_{sgd,momentum,adam}`` (``csrc/optim.hip``);
CPU tensors use the vectorised PyTorch reference below (same math).

``dyn`` (optional) is a device float32 tensor ``[lr, lr_t, grad_scale]`` the
kernels read instead of their scalar arguments, so a hipGraph-captured step
(:mod:`mdtf.train.graph`) picks up per-step values without re-capture.
"""
import math

import torch

from . import _native

_native.register("mdtf_fused_sgd", [_native.L, _native.P, _native.P, _native.P,
                                    _native.F, _native.F, _native.F, _native.P, _native.P])
_native.register("mdtf_fused_momentum", [_native.L, _native.P, _native.P, _native.P, _native.P,
                                         _native.F, _native.F, _native.F, _native.F, _native.I, _native.P, _native.P])
_native.register("mdtf_fused_adam", [_native.L, _native.P, _native.P, _native.P, _native.P, _native.P,
                                     _native.F, _native.F, _native.F, _native.F, _native.F, _native.F,
                                     _native.F, _native.I, _native.P, _native.P])


def _shadow_code(shadow):
    return shadow


def _native_ok(master):
    return master.is_cuda and _native.mode() != "torch" and _native.use_native(master)


def _dyn_scalars(dyn, lr, lr_t, grad_scale):
    if dyn is None:
        return lr, lr_t, grad_scale
    d = dyn.tolist()
    return d[0], d[1], d[2]


def sgd_(master, grad, shadow, lr, grad_scale=1.0, weight_decay=0.0, dyn=None):
    """``w -= lr * (g*scale + wd*w)``; refresh ``shadow`` if given."""
    if _native_ok(master):
        n = master.numel()
        _native.check(_native.fn("mdtf_fused_sgd")(
            n, _native.ptr(master), _native.ptr(grad), _native.ptr(shadow),
            float(lr), float(grad_scale), float(weight_decay), _native.ptr(dyn), _native.stream_ptr()), "fused_sgd")
        return
    lr, _, grad_scale = _dyn_scalars(dyn, lr, lr, grad_scale)
    g = grad.float() * grad_scale
    if weight_decay:
        g = g + weight_decay * master
    master.sub_(lr * g)
    if shadow is not None:
        shadow.copy_(master)


def momentum_(master, grad, accum, shadow, lr, momentum, grad_scale=1.0, weight_decay=0.0, nesterov=False,
              dyn=None):
    """TF MomentumOptimizer: ``a = m*a + g``; ``w -= lr*a`` (nesterov: ``lr*(g + m*a)``)."""
    if _native_ok(master):
        n = master.numel()
        _native.check(_native.fn("mdtf_fused_momentum")(
            n, _native.ptr(master), _native.ptr(grad), _native.ptr(accum), _native.ptr(shadow),
            float(lr), float(momentum), float(grad_scale), float(weight_decay), int(bool(nesterov)),
            _native.ptr(dyn), _native.stream_ptr()), "fused_momentum")
        return
    lr, _, grad_scale = _dyn_scalars(dyn, lr, lr, grad_scale)
    g = grad.float() * grad_scale
    if weight_decay:
        g = g + weight_decay * master
    accum.mul_(momentum).add_(g)
    if nesterov:
        master.sub_(lr * (g + momentum * accum))
    else:
        master.sub_(lr * accum)
    if shadow is not None:
        shadow.copy_(master)


def adam_lr_t(lr, beta1, beta2, step, bias_correction=True):
    """TF Adam's step size with the bias correction folded in (``step`` counts from 1)."""
    if not bias_correction:
        return lr
    return lr * math.sqrt(1.0 - beta2 ** step) / (1.0 - beta1 ** step)


def adam_(master, grad, m, v, shadow, lr, beta1, beta2, epsilon, step, grad_scale=1.0, weight_decay=0.0,
          decoupled=False, bias_correction=True, dyn=None):
    """Adam (TF form: bias correction folded into lr, eps added outside sqrt).

    ``decoupled=True`` gives AdamW/BERT's AdamWeightDecay:
    ``w -= lr * (m_hat/(sqrt(v_hat)+eps) + wd*w)``; otherwise ``wd`` is L2
    (added to the gradient).
    """
    lr_t = adam_lr_t(lr, beta1, beta2, step, bias_correction)
    if _native_ok(master):
        n = master.numel()
        _native.check(_native.fn("mdtf_fused_adam")(
            n, _native.ptr(master), _native.ptr(grad), _native.ptr(m), _native.ptr(v), _native.ptr(shadow),
            float(lr), float(lr_t), float(beta1), float(beta2), float(epsilon), float(grad_scale),
            float(weight_decay), int(bool(decoupled)), _native.ptr(dyn), _native.stream_ptr()), "fused_adam")
        return
    lr, lr_t, grad_scale = _dyn_scalars(dyn, lr, lr_t, grad_scale)
    g = grad.float() * grad_scale
    if weight_decay and not decoupled:
        g = g + weight_decay * master
    m.mul_(beta1).add_(g, alpha=1 - beta1)
    v.mul_(beta2).addcmul_(g, g, value=1 - beta2)
    upd = lr_t * m / (v.sqrt() + epsilon)
    if weight_decay and decoupled:
        upd = upd + lr * weight_decay * master
    master.sub_(upd)
    if shadow is not None:
        shadow.copy_(master)


_native.register("mdtf_fused_apply_multi", [_native.I, _native.L, _native.P, _native.P, _native.P, _native.P, _native.P,
                                            _native.P, _native.P, _native.I, _native.I, _native.F, _native.F,
                                            _native.F, _native.F, _native.F, _native.F, _native.I, _native.P])
MAX_MULTI = 8
_KIND = {"sgd": 0, "momentum": 1, "adam": 2}


def apply_multi_(kind, master, grads, s1, s2, shadow, lrs, lr_ts, momentum=0.0, beta1=0.9, beta2=0.999,
                 epsilon=1e-8, grad_scale=1.0, weight_decay=0.0, flag=False):
    """``len(grads)`` (<= 8) SEQUENTIAL updates of one flat group in one pass: update i applies ``grads[i]``
    (bf16 wire or fp32) with ``lrs[i]`` / ``lr_ts[i]``.  Equals that many single-update launches in order
    (the async parameter server applies every gradient that arrived since its last apply this way).
    ``flag``: nesterov (momentum) / decoupled weight decay (adam)."""
    k = len(grads)
    assert 1 <= k <= MAX_MULTI and len(lrs) == k and len(lr_ts) == k
    if _native_ok(master) and all(g.dtype == grads[0].dtype for g in grads):
        import ctypes
        gp = (ctypes.c_void_p * k)(*[g.data_ptr() for g in grads])
        fl = (ctypes.c_float * k)(*[float(x) for x in lrs])
        ft = (ctypes.c_float * k)(*[float(x) for x in lr_ts])
        _native.check(_native.fn("mdtf_fused_apply_multi")(
            _KIND[kind], master.numel(), _native.ptr(master), _native.ptr(s1), _native.ptr(s2), _native.ptr(shadow),
            ctypes.cast(gp, ctypes.c_void_p), ctypes.cast(fl, ctypes.c_void_p), ctypes.cast(ft, ctypes.c_void_p), k,
            int(grads[0].dtype == torch.bfloat16), float(momentum), float(beta1), float(beta2), float(epsilon),
            float(grad_scale), float(weight_decay), int(bool(flag)), _native.stream_ptr()), "fused_apply_multi")
        return
    for g, lr, lr_t in zip(grads, lrs, lr_ts):
        g = g.float() * grad_scale
        if kind == "adam":
            if weight_decay and not flag:
                g = g + weight_decay * master
            s1.mul_(beta1).add_(g, alpha=1 - beta1)
            s2.mul_(beta2).addcmul_(g, g, value=1 - beta2)
            upd = lr_t * s1 / (s2.sqrt() + epsilon)
            if weight_decay and flag:
                upd = upd + lr * weight_decay * master
            master.sub_(upd)
            continue
        if weight_decay:
            g = g + weight_decay * master
        if kind == "momentum":
            s1.mul_(momentum).add_(g)
            master.sub_(lr * (g + momentum * s1) if flag else lr * s1)
        else:
            master.sub_(lr * g)
    if shadow is not None:
        shadow.copy_(master)
