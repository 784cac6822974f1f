"""Conv time vs reduction length K at fixed output (1x1 conv M=50176, N=1024): separates the per-tile fixed
cost (fill latency, copy-out) from the K loop."""
import os, sys, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench.conv_autotune import timeit
from mdtf.ops import conv as C
dev="cuda"
print("1x1 conv M=50176 N=1024, no stats: v2 128x128s2 | v2 128x128s3 | v3 256x256s2 | v3 256x128s3")
for K in (64, 128, 256, 512, 1024, 2048):
    x=torch.randn(256,14,14,K,device=dev).bfloat16(); w=(torch.randn(1,1,K,1024,device=dev)*0.05).bfloat16()
    r=[]
    for bm,bn,st,v in ((128,128,2,2),(128,128,3,2),(256,256,2,3),(256,128,3,3)):
        try:
            t=timeit(lambda: C.mdtf_fwd(x,w,(14,14),(1,1),(0,0,0,0),(1,1),bm,bn,None,v,st),10)
        except RuntimeError:
            t=float('nan')
        r.append(t)
    fl=2*50176*K*1024
    print("K=%5d  "%K + "  ".join("%.3f ms (%4.0f TF/s)"%(t, fl/t/1e9) for t in r))
