"""Run a few representative conv kernels repeatedly (for rocprofv3 --pmc)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from mdtf.ops import conv as C
dev = "cuda"
torch.manual_seed(0)
cases = [(256, 14, 14, 256, 3, 256), (256, 56, 56, 64, 1, 256)]
for (n, h, w, c, k, co) in cases:
    x = torch.randn(n, h, w, c, device=dev).bfloat16()
    wt = (torch.randn(k, k, c, co, device=dev) * 0.05).bfloat16()
    p = (k // 2,) * 4
    dy = torch.randn(n, h, w, co, device=dev).bfloat16()
    out = torch.zeros(k, k, c, co, device=dev)
    for _ in range(10):
        C.mdtf_fwd(x, wt, (h, w), (1, 1), p, (1, 1), 128, 128, None, 2, 2)
        C.mdtf_dgrad(dy, wt, x.shape, (1, 1), p, (1, 1), 128, 128, 2, 2)
        C.mdtf_wgrad(x, dy, wt.shape, (1, 1), p, (1, 1), 128, 128, 0, out=out, ver=2, stages=2)
torch.cuda.synchronize()
print("ok")
