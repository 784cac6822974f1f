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
"""
import math

import torch

from . import _native

_native.register("mdtf_fused_sgd", [_native.L, _native.P, _native.P, _native.P,
                                    _native.F, _native.F, _native.F, _native.P])
_native.register("mdtf_fused_momentum", [_native.L, _native.P, _native.P, _native.P, _native.P,
                                         _native.F, _native.F, _native.F, _native.F, _native.I, _native.P])
_native.register("mdtf_fused_adam", [_native.L, _native.P, _native.P, _native.P, _native.P, _native.P,
                                     _native.F, _native.F, _native.F, _native.F, _native.F, _native.F,
                                     _native.F, _native.F, _native.I, _native.P])


def _shadow_code(shadow):
    return shadow


def _native_ok(master):
    return master.is_cuda and _native.mode() != "torch" and _native.use_native(master)


def sgd_(master, grad, shadow, lr, grad_scale=1.0, weight_decay=0.0):
    """``w -= lr * (g*scale + wd*w)``; refresh ``shadow`` if given."""
    if _native_ok(master):
        n = master.numel()
        _native.check(_native.fn("mdtf_fused_sgd")(
            n, _native.ptr(master), _native.ptr(grad), _native.ptr(shadow),
            float(lr), float(grad_scale), float(weight_decay), _native.stream_ptr()), "fused_sgd")
        return
    g = grad.float() * grad_scale
    if weight_decay:
        g = g + weight_decay * master
    master.sub_(lr * g)
    if shadow is not None:
        shadow.copy_(master)


def momentum_(master, grad, accum, shadow, lr, momentum, grad_scale=1.0, weight_decay=0.0, nesterov=False):
    """TF MomentumOptimizer: ``a = m*a + g``; ``w -= lr*a`` (nesterov: ``lr*(g + m*a)``)."""
    if _native_ok(master):
        n = master.numel()
        _native.check(_native.fn("mdtf_fused_momentum")(
            n, _native.ptr(master), _native.ptr(grad), _native.ptr(accum), _native.ptr(shadow),
            float(lr), float(momentum), float(grad_scale), float(weight_decay), int(bool(nesterov)),
            _native.stream_ptr()), "fused_momentum")
        return
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


def adam_(master, grad, m, v, shadow, lr, beta1, beta2, epsilon, step, grad_scale=1.0, weight_decay=0.0,
          decoupled=False, bias_correction=True):
    """Adam (TF form: bias correction folded into lr, eps added outside sqrt).

    ``decoupled=True`` gives AdamW/BERT's AdamWeightDecay:
    ``w -= lr * (m_hat/(sqrt(v_hat)+eps) + wd*w)``; otherwise ``wd`` is L2
    (added to the gradient).
    """
    if bias_correction:
        bc1 = 1.0 - beta1 ** step
        bc2 = 1.0 - beta2 ** step
        lr_t = lr * math.sqrt(bc2) / bc1
    else:
        lr_t = lr
    if _native_ok(master):
        n = master.numel()
        _native.check(_native.fn("mdtf_fused_adam")(
            n, _native.ptr(master), _native.ptr(grad), _native.ptr(m), _native.ptr(v), _native.ptr(shadow),
            float(lr), float(lr_t), float(beta1), float(beta2), float(epsilon), float(grad_scale),
            float(weight_decay), 0.0, int(bool(decoupled)), _native.stream_ptr()), "fused_adam")
        return
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
