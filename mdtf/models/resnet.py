"""ResNet v1.5 (50 / 101 / 152) in NHWC on mdtf kernels.

BASELINE configs: "ResNet-50 bf16 single-worker", "ResNet-50 sync-SGD 8
workers", "ResNet-152 async parameter-server" (BASELINE.json).  Architecture:
TF-official ResNet v1.5 (stride on the 3x3 conv of the bottleneck), 7x7/2 stem,
3x3/2 max-pool, bottleneck stages, global average pool, 1000-way dense.

Every conv is followed by a fused BatchNorm(+residual)(+ReLU) kernel
(``tools.conv_bn``); the last BN of each block carries the residual add and
ReLU, so a bottleneck block is 3-4 conv launches + 3 BN launches.  Variable
names follow TF-slim style scopes (``resnet_v1_50/block1/unit_1/conv1/weights``).
"""
import os

import torch

from ..layers import tools
from ..ops import nn as ops
from ..runtime.model import Loss, Model
from ..train import variables as V

DEPTHS = {18: None, 50: [3, 4, 6, 3], 101: [3, 4, 23, 3], 152: [3, 8, 36, 3], 200: [3, 24, 36, 3]}



# MDTF_PROJ_LATE=1: run the projection shortcut's conv after conv2, so its backward runs before conv1's and its data
# gradient can be fused into conv1's (ops.actsink deferral + mdtf_conv_ws_dual).  Off by default: measured neutral
# in the step (+0.1 %, profiles/ab_r5.md) -- the split order (conv1 writes, the projection accumulates with the
# statistics, the zero classes only read) already moves little more than the fused pass would.
PROJ_LATE = os.environ.get("MDTF_PROJ_LATE", "0") == "1"

class ResNet(Model):
    def __init__(self, depth=50, num_classes=1000, zero_init_residual=True, bn_decay=0.9, bn_epsilon=1e-5,
                 width=64):
        if DEPTHS.get(depth) is None:
            raise ValueError("unsupported ResNet depth %d" % depth)
        self.depth = depth
        self.blocks = DEPTHS[depth]
        self.num_classes = num_classes
        self.zero_init_residual = zero_init_residual
        self.bn_decay = bn_decay
        self.bn_epsilon = bn_epsilon
        self.width = width
        self.name = "resnet_v1_%d" % depth

    def _bottleneck(self, x, filters, stride, name, training):
        kw = dict(training=training, bn_decay=self.bn_decay, bn_epsilon=self.bn_epsilon)
        with V.variable_scope(name):
            proj = stride != 1 or x.shape[-1] != 4 * filters
            if proj and not PROJ_LATE:
                shortcut = tools.conv_bn("shortcut", x, 4 * filters, 1, stride, relu=False, defer=True, **kw)
            elif proj:
                # GPU training: its BN is applied inside conv3's residual BN pass (ops.bn.DeferredBN).  The
                # variables are created first (the checkpoint / initialisation order); the conv itself runs
                # after conv2, so autograd runs its backward BEFORE conv1's: the strided projection's data
                # gradient is the first contribution to x's gradient and can be deferred into conv1's
                # (ops.actsink, one fused pass over the block input's gradient)
                sc_vars = tools.conv_bn_variables("shortcut", x, 4 * filters, 1, **kw)
            y = tools.conv_bn("conv1", x, filters, 1, 1, relu=True, **kw)
            # (conv3 is its output's only reader: it may apply this BN + ReLU to its operand, ops.bn ON_CONSUMER)
            y = tools.conv_bn("conv2", y, filters, 3, stride, relu=True, on_consumer=True, **kw)
            if proj and PROJ_LATE:
                shortcut = tools.conv_bn_apply(x, sc_vars, 1, stride, relu=False, defer=True, **kw)
            elif not proj:
                shortcut = x
            y = tools.conv_bn("conv3", y, 4 * filters, 1, 1, relu=True, residual=shortcut,
                              zero_gamma=self.zero_init_residual, **kw)
        return y

    def inference(self, input_data, training=None):
        from ..train.step import is_training
        training = is_training() if training is None else training
        store = V.get_store()
        x = input_data
        if store.compute_dtype is not None and x.dtype != store.compute_dtype:
            x = x.to(store.compute_dtype)
        with V.variable_scope(self.name):
            # stem conv -> BN -> ReLU -> 3x3/2 max pool (BN + ReLU + pool one pass on the GPU)
            x = tools.conv_bn("conv1", x, self.width, 7, 2, relu=True, training=training,
                              bn_decay=self.bn_decay, bn_epsilon=self.bn_epsilon, pool=(3, 2, "SAME"))
            for s, n in enumerate(self.blocks):
                filters = self.width * (2 ** s)
                for u in range(n):
                    stride = 2 if (u == 0 and s > 0) else 1
                    x = self._bottleneck(x, filters, stride, "block%d/unit_%d" % (s + 1, u + 1), training)
            x = ops.global_avg_pool(x)
            logits = tools.dense("logits", x, self.num_classes,
                                 initializer=V.random_normal_initializer(stddev=0.01))
        return logits


class ResNet50(ResNet):
    def __init__(self, **kw):
        super(ResNet50, self).__init__(50, **kw)


class ResNet152(ResNet):
    def __init__(self, **kw):
        super(ResNet152, self).__init__(152, **kw)


class SoftmaxCrossEntropyLoss(Loss):
    """Mean sparse softmax cross entropy (fp32), optional label smoothing."""

    def __init__(self, label_smoothing=0.0):
        self.label_smoothing = label_smoothing

    def loss(self, predict, ground_truth):
        if self.label_smoothing:
            n = predict.shape[-1]
            logp = torch.log_softmax(predict.float(), -1)
            onehot = torch.nn.functional.one_hot(ground_truth.long(), n).float()
            target = onehot * (1 - self.label_smoothing) + self.label_smoothing / n
            return -(target * logp).sum(-1).mean()
        return ops.sparse_softmax_cross_entropy_with_logits(ground_truth, predict).mean()
