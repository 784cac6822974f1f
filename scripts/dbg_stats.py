import os, sys, torch
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "/root/repo"))
os.environ["MDTF_CONV"] = "mdtf"
from mdtf.ops import conv as C, nn as ops
def rel(a,b): return ((a.float().cpu()-b.float().cpu()).norm()/b.float().cpu().norm()).item()
torch.manual_seed(0)
shape=(8,14,14,64); k=1; co=256
x = torch.randn(shape); w = torch.randn(k,k,64,co)*0.125; g=torch.rand(co)+0.5; b=torch.randn(co)*0.1
r = torch.randn(8,14,14,co)
for relu in (False, True):
    for res in (False, True):
        for use_stats in (True, False):
            outs={}
            for dev,dt in (("cuda",torch.bfloat16),("cpu",torch.float32)):
                mm=torch.zeros(co,device=dev); mv=torch.ones(co,device=dev)
                rr = r.to(dev).to(dt) if res else None
                if use_stats or dev=="cpu":
                    y = ops.conv_bn(x.to(dev).to(dt), w.to(dev).to(dt), g.to(dev), b.to(dev), mm, mv, 1, "SAME", True, 0.9, 1e-5, relu, rr)
                else:
                    yc = ops.conv2d(x.to(dev).to(dt), w.to(dev).to(dt), 1, "SAME")
                    y = ops.batch_norm(yc, g.to(dev), b.to(dev), mm, mv, True, 0.9, 1e-5, relu, rr)
                outs[dev]=(y.detach(), mm, mv)
            print("relu",relu,"res",res,"stats",use_stats,"y",rel(outs["cuda"][0],outs["cpu"][0]),"mm",rel(outs["cuda"][1],outs["cpu"][1]),"mv",rel(outs["cuda"][2],outs["cpu"][2]))
