#!/usr/bin/env python
"""One eager ResNet-50 training step (batch 32) on the GPU with MDTF_BN_TRACE=1: lists every BatchNorm backward
whose statistics did NOT come from the completing conv's dgrad epilogue (those pay a separate reduce pass)."""
import collections
import os
import sys

os.environ["MDTF_BN_TRACE"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import mdtf  # noqa: E402
from mdtf.models import ResNet, SoftmaxCrossEntropyLoss  # noqa: E402
from mdtf.ops import bn  # noqa: E402
from mdtf.runtime import Net, Tower  # noqa: E402
from mdtf.train import variables as V  # noqa: E402

store = V.get_store()
store.device = torch.device("cuda", 0)
store.compute_dtype = torch.bfloat16
xp = mdtf.placeholder(torch.float32, [None, 224, 224, 3])
yp = mdtf.placeholder(torch.int64, [None])
opt = mdtf.train.MomentumOptimizer(0.1, 0.9)
tg = []
t = Tower(Net(ResNet(50, num_classes=1000)), "tower_0/", tg, xp, yp, SoftmaxCrossEntropyLoss(), opt, batch_size=32)
_, loss, _ = t.process()
op = opt.apply_gradients(Tower.average_gradients(tg), global_step=mdtf.train.get_or_create_global_step())
sess = mdtf.train.MonitoredTrainingSession(log_step_count_steps=0)
x = torch.randn(32, 224, 224, 3)
y = torch.randint(0, 1000, (32,))
for _ in range(2):
    bn.BWD_TRACE.clear()
    sess.run([op, loss], feed_dict={xp: x, yp: y})
torch.cuda.synchronize()
c = collections.Counter(w for _, _, w in bn.BWD_TRACE)
print("BN backward statistics source:", dict(c))
for shp, res, why in bn.BWD_TRACE:
    if why != "fused":
        print("  ", shp, "residual" if res else "", why)
