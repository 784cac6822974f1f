"""Layer toolkit — the ``distribute_tools.py`` API on MI355X kernels.

Every function keeps the reference's name, arguments, variable names
(``weights``/``biases``/``weights_nonacti``/``biases_nonacti`` under the
``layer_name`` scope, SURVEY §9.5 — these become checkpoint tensor names) and
TF layouts (NHWC activations, HWIO filters).  Compute runs on the fused HIP
kernels of :mod:`mdtf.ops` (conv + bias + ReLU in one epilogue, BN statistics +
normalise + ReLU (+ residual) fused, ...).

Fixes: ``norm`` returns the LRN output (Q17); ``batch_norm`` is a
standard per-channel BN with affine parameters and moving statistics (Q18) —
``batch_norm(x, legacy=True)`` keeps the reference's batch-axis-only,
affine-free behaviour.
"""
import torch

from ..config.flags import FLAGS
from ..ops import nn as ops
from ..train import variables as V


def _dtype():
    return torch.float32  # masters are fp32; FLAGS.use_fp16 selects bf16 *compute* (see Train)


def _variable_on_cpu(name, shape, initializer):
    """Create/reuse a variable (``distribute_tools.py:24-38``).

    The name is historical: variables live in the HBM of the rank that owns
    them; the fp16 flag selects reduced-precision compute, not storage.
    """
    return V.get_variable(name, shape, dtype=_dtype(), initializer=initializer)


def _variable_with_weight_decay(name, shape, stddev, wd):
    """Truncated-normal variable; adds ``wd * l2_loss(var)`` to 'losses' (``:41-66``)."""
    var = _variable_on_cpu(name, shape, V.truncated_normal_initializer(stddev=stddev))
    if wd is not None and wd != 0.0:
        store = V.get_store()
        scope = V.get_variable_scope().name
        full = "%s/%s" % (scope, name) if scope else name
        V.add_to_collection("losses", ops.l2_loss(store.vars[full].read(store.compute_dtype)) * wd)
    return var


def _strides(stride):
    return stride


def conv(layer_name, x, in_channels, out_channels, kernel_size=(3, 3), stride=(1, 1, 1, 1)):
    """conv (SAME) + bias + ReLU in one fused kernel (``distribute_tools.py:69-79``)."""
    with V.variable_scope(layer_name):
        return _conv_body(x, in_channels, out_channels, kernel_size, stride)


def conv_eval(layer_name, x, in_channels, out_channels, kernel_size=(3, 3), stride=(1, 1, 1, 1)):
    """``conv`` with AUTO_REUSE (``:81-91``)."""
    with V.variable_scope(layer_name, reuse=V.AUTO_REUSE):
        return _conv_body(x, in_channels, out_channels, kernel_size, stride)


def _conv_body(x, in_channels, out_channels, kernel_size, stride):
    w = _variable_with_weight_decay('weights', [kernel_size[0], kernel_size[1], in_channels, out_channels],
                                    stddev=5e-2, wd=0.0)
    b = _variable_on_cpu('biases', [out_channels], V.constant_initializer(0.0))
    return ops.conv2d(x, w, _strides(stride), "SAME", bias=b, act="relu")


def conv_nonacti(layer_name, x, in_channels, out_channels, kernel_size=(3, 3), stride=(1, 1, 1, 1)):
    """conv + bias, no activation; Xavier init (``:93-105``)."""
    with V.variable_scope(layer_name):
        return _conv_nonacti_body(x, in_channels, out_channels, kernel_size, stride)


def conv_nonacti_eval(layer_name, x, in_channels, out_channels, kernel_size=(3, 3), stride=(1, 1, 1, 1)):
    with V.variable_scope(layer_name, reuse=V.AUTO_REUSE):
        return _conv_nonacti_body(x, in_channels, out_channels, kernel_size, stride)


def _conv_nonacti_body(x, in_channels, out_channels, kernel_size, stride):
    w = V.get_variable('weights_nonacti', [kernel_size[0], kernel_size[1], in_channels, out_channels],
                       initializer=V.xavier_initializer())
    b = V.get_variable('biases_nonacti', [out_channels], initializer=V.constant_initializer(0.0))
    return ops.conv2d(x, w, _strides(stride), "SAME", bias=b)


def acti_layer(x):
    """ReLU (``:123-128``)."""
    return ops.relu(x)


def deconv(layer_name, x, in_channels, out_channels, output_shape=(32, 224, 224, 64), kernel_size=(3, 3),
           stride=(1, 1, 1, 1)):
    """Transposed conv, no bias (``:131-143``).

    As in the reference the filter is created ``[kh, kw, in_channels, out_channels]``
    and interpreted with TF's transposed-conv layout ``[kh, kw, C_out_of_op, C_in_of_op]``.
    """
    with V.variable_scope(layer_name):
        return _deconv_body(x, in_channels, out_channels, output_shape, kernel_size, stride)


def deconv_eval(layer_name, x, in_channels, out_channels, output_shape=(32, 224, 224, 64), kernel_size=(3, 3),
                stride=(1, 1, 1, 1)):
    with V.variable_scope(layer_name, reuse=V.AUTO_REUSE):
        return _deconv_body(x, in_channels, out_channels, output_shape, kernel_size, stride)


def _deconv_body(x, in_channels, out_channels, output_shape, kernel_size, stride):
    w = V.get_variable('weights', [kernel_size[0], kernel_size[1], in_channels, out_channels],
                       initializer=V.xavier_initializer())
    return ops.conv2d_transpose(x, w, output_shape, _strides(stride), "SAME")


def pool(layer_name, x, kernel=(1, 2, 2, 1), stride=(1, 2, 2, 1), is_max_pool=True):
    """2x2/2 SAME max (default) or average pool (``:160-165``)."""
    if is_max_pool:
        return ops.max_pool(x, kernel, stride, "SAME", name=layer_name)
    return ops.avg_pool(x, kernel, stride, "SAME", name=layer_name)


def batch_norm(x, legacy=False, training=True, decay=0.9, epsilon=1e-3, relu=False, residual=None,
               name="batch_norm"):
    """Batch normalisation.

    ``legacy=True`` reproduces ``distribute_tools.py:168-180`` exactly
    (moments over axis 0 only, no offset/scale, no moving statistics).
    Otherwise: per-channel BN with ``gamma``/``beta`` and moving statistics,
    fused with optional residual add and ReLU.
    """
    if legacy:
        mean, var = ops.moments(x, [0])
        return ops.batch_normalization(x, mean, var, None, None, epsilon)
    c = x.shape[-1]
    with V.variable_scope(name, reuse=V.AUTO_REUSE if V.get_store().frozen else None):
        gamma = V.get_variable('gamma', [c], initializer=V.constant_initializer(1.0), keep_fp32=True)
        beta = V.get_variable('beta', [c], initializer=V.constant_initializer(0.0), keep_fp32=True)
        mm = V.get_variable('moving_mean', [c], initializer=V.constant_initializer(0.0), trainable=False)
        mv = V.get_variable('moving_variance', [c], initializer=V.constant_initializer(1.0), trainable=False)
    return ops.batch_norm(x, gamma, beta, mm, mv, training, decay, epsilon, relu, residual)


def norm(name, x, lsize=4):
    """Local response normalisation; returns the LRN output (fix for SURVEY Q17)."""
    return ops.lrn(x, lsize, bias=1.0, alpha=0.001 / 9.0, beta=0.75, name=name)


def FC_layer(layer_name, x, out_nodes, act="relu"):
    """Flatten + matmul + bias + ReLU, Xavier init (``:190-208``)."""
    if x.dim() == 4:
        size = x.shape[1] * x.shape[2] * x.shape[3]
    else:
        size = x.shape[-1]
    with V.variable_scope(layer_name):
        w = V.get_variable('weights', [size, out_nodes], initializer=V.xavier_initializer())
        b = V.get_variable('biases', [out_nodes], initializer=V.constant_initializer(0.0))
        flat_x = x.reshape(-1, size)
        return ops.dense(flat_x, w, b, act=act)


def weight(kernel_shape, is_uniform=True):
    """Bare Xavier ``weights`` variable in the current scope (``:211-216``)."""
    return V.get_variable('weights', kernel_shape, initializer=V.xavier_initializer(uniform=is_uniform))


def bias(bias_shape):
    """Bare zero-initialised ``biases`` variable (``:219-224``)."""
    return V.get_variable('biases', bias_shape, initializer=V.constant_initializer(0.0))


# ---------------------------------------------------------------------------
# Layers used by the model zoo (ResNet / BERT), same variable conventions.
# ---------------------------------------------------------------------------


def conv_bn(layer_name, x, out_channels, kernel_size=3, stride=1, relu=True, residual=None, training=True,
            bn_decay=0.9, bn_epsilon=1e-5, zero_gamma=False, padding=None, defer=False, pool=None, on_consumer=False):
    """conv (no bias) → BN (→ +residual) (→ ReLU), ResNet v1.5 building unit.

    Stride>1 convs use TF-official "fixed padding" (symmetric ``(k-1)//2``).  ``defer``: the BN may be
    returned unapplied (``ops.bn.DeferredBN``) for the residual BN that adds it to apply (GPU training).
    ``pool = (ksize, stride, padding)``: a max pool after the ReLU (fused with the BN on the GPU).
    ``on_consumer``: the output's only reader is a 1x1 conv, which may apply the BN + ReLU itself (GPU training).
    """
    variables = conv_bn_variables(layer_name, x, out_channels, kernel_size, zero_gamma=zero_gamma)
    return conv_bn_apply(x, variables, kernel_size, stride, relu, residual, training, bn_decay, bn_epsilon, padding,
                         defer, pool, on_consumer)


def conv_bn_apply(x, variables, kernel_size=3, stride=1, relu=True, residual=None, training=True, bn_decay=0.9,
                  bn_epsilon=1e-5, padding=None, defer=False, pool=None, on_consumer=False):
    """:func:`conv_bn` on variables already made by :func:`conv_bn_variables`."""
    k = kernel_size
    if padding is None:
        padding = "SAME" if stride == 1 else ((k - 1) // 2, (k - 1) // 2)
    w, gamma, beta, mm, mv = variables
    return ops.conv_bn(x, w, gamma, beta, mm, mv, stride, padding, training, bn_decay, bn_epsilon, relu, residual,
                       defer=defer, pool=pool, on_consumer=on_consumer)


def conv_bn_variables(layer_name, x, out_channels, kernel_size=3, zero_gamma=False, **unused):
    """The variables of :func:`conv_bn` (created on first use, reused after): weights, gamma, beta, moving
    mean / variance."""
    k = kernel_size
    with V.variable_scope(layer_name):
        w = V.get_variable('weights', [k, k, x.shape[-1], out_channels], initializer=V.variance_scaling_initializer())
        c = out_channels
        gamma = V.get_variable('BatchNorm/gamma', [c], initializer=V.constant_initializer(0.0 if zero_gamma else 1.0),
                               keep_fp32=True)
        beta = V.get_variable('BatchNorm/beta', [c], initializer=V.constant_initializer(0.0), keep_fp32=True)
        mm = V.get_variable('BatchNorm/moving_mean', [c], initializer=V.constant_initializer(0.0), trainable=False)
        mv = V.get_variable('BatchNorm/moving_variance', [c], initializer=V.constant_initializer(1.0),
                            trainable=False)
    return w, gamma, beta, mm, mv


def dense(layer_name, x, out_features, act=None, initializer=None):
    with V.variable_scope(layer_name):
        w = V.get_variable('kernel', [x.shape[-1], out_features],
                           initializer=initializer or V.truncated_normal_initializer(stddev=0.02))
        b = V.get_variable('bias', [out_features], initializer=V.constant_initializer(0.0))
        shp = x.shape
        y = ops.dense(x.reshape(-1, shp[-1]), w, b, act=act)
        return y.reshape(*shp[:-1], out_features)


def layer_norm(layer_name, x, epsilon=1e-12):
    with V.variable_scope(layer_name):
        g = V.get_variable('gamma', [x.shape[-1]], initializer=V.constant_initializer(1.0), keep_fp32=True)
        b = V.get_variable('beta', [x.shape[-1]], initializer=V.constant_initializer(0.0), keep_fp32=True)
        return ops.layer_norm(x, g, b, epsilon)
