import os, sys, torch
root = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path.insert(0, root); sys.path.insert(0, os.path.join(root, "tests"))
import mdtf
from mdtf.layers import tools
from mdtf.ops import nn as ops
from mdtf.runtime import Model, Net, Tower
from mdtf.models import SoftmaxCrossEntropyLoss
from mdtf.train import step as S, variables as V
def rel(a,b): return ((a.float().cpu()-b.float().cpu()).norm()/(b.float().cpu().norm()+1e-12)).item()

class Tiny(Model):
    def __init__(self, variant): self.variant = variant
    def inference(self, x):
        store = V.get_store()
        if store.compute_dtype is not None: x = x.to(store.compute_dtype)
        if self.variant >= 1:
            x = tools.conv_bn("c1", x, 64, 3, 1, relu=True)
        if self.variant >= 2:
            x = ops.max_pool(x, 3, 2, "SAME")
        if self.variant >= 3:
            s = x
            y = tools.conv_bn("c2", x, 64, 1, 1, relu=True)
            x = tools.conv_bn("c3", y, 64, 3, 1, relu=True, residual=s)
        x = ops.global_avg_pool(x)
        return tools.dense("logits", x, 16)

def step(dev, dt, variant, x, y):
    V.reset_default_graph(); S.reset()
    store = V.get_store(); store.device = torch.device(dev); store.compute_dtype = dt
    store.generator.manual_seed(123)
    xp = mdtf.placeholder(torch.float32, [None]+list(x.shape[1:])); yp = mdtf.placeholder(torch.int64, [None])
    opt = mdtf.train.GradientDescentOptimizer(0.1); tg=[]
    t = Tower(Net(Tiny(variant)), "tower_0/", tg, xp, yp, SoftmaxCrossEntropyLoss(), opt, batch_size=x.shape[0])
    _, loss, _ = t.process()
    op = opt.apply_gradients(Tower.average_gradients(tg), global_step=mdtf.train.get_or_create_global_step())
    sess = mdtf.train.MonitoredTrainingSession(log_step_count_steps=0)
    _, lv = sess.run([op, loss], feed_dict={xp: x, yp: y})
    return float(lv), {v.name: v.grad.detach().float().cpu().clone() for v in store.trainable_variables()}

torch.manual_seed(0)
x = torch.randn(16, 16, 16, 8); y = torch.randint(0, 16, (16,))
for mode in ("mdtf", "miopen"):
    os.environ["MDTF_CONV"] = mode
    for variant in (0, 1, 2, 3):
        lc, gc = step("cpu", None, variant, x, y)
        lg, gg = step("cuda", torch.bfloat16, variant, x, y)
        print(mode, "variant", variant, "loss", lc, lg, {k: round(rel(gg[k], gc[k]), 4) for k in gc})
