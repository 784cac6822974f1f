"""LeNet for MNIST (BASELINE config 1: 1-ps/1-worker localhost ClusterSpec on CPU).

Built purely from the reference toolkit API (``tools.conv``, ``tools.pool``,
``tools.FC_layer``), so it also exercises the variable naming conventions
(``conv1/weights``, ``fc1/biases``...) and the weight-decay loss collection.
"""
from ..layers import tools
from ..runtime.model import Model
from ..train import variables as V


class LeNet(Model):
    def __init__(self, num_classes=10, weight_decay=None):
        self.num_classes = num_classes
        self.weight_decay = weight_decay

    def inference(self, input_data):
        x = input_data
        store = V.get_store()
        if store.compute_dtype is not None:
            x = x.to(store.compute_dtype)
        if x.dim() == 3:
            x = x.unsqueeze(-1)
        x = tools.conv("conv1", x, x.shape[-1], 32, kernel_size=[5, 5])
        x = tools.pool("pool1", x)
        x = tools.conv("conv2", x, 32, 64, kernel_size=[5, 5])
        x = tools.pool("pool2", x)
        x = tools.FC_layer("fc1", x, 512)
        logits = tools.FC_layer("fc2", x, self.num_classes, act=None)
        if self.weight_decay:
            from ..ops import nn as ops
            for name in ("fc1/weights", "fc2/weights"):
                V.add_to_collection("losses", ops.l2_loss(store.vars[name].read(store.compute_dtype))
                                    * self.weight_decay)
        return logits
