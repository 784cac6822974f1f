import torch, sys
sys.path.insert(0, '.')
from mdtf.ops import conv as C
DEV = 'cuda'
torch.manual_seed(0)
x = torch.randn(3, 17, 15, 64, device=DEV).bfloat16()
wt = (torch.randn(1, 1, 64, 192, device=DEV) / 8).bfloat16()
y = C.pp_fwd(x, wt, (17, 15), (1, 1), (0,) * 4, (1, 1), 4).float().reshape(-1, 192)
X = x.float().reshape(-1, 64)
Beff = torch.linalg.lstsq(X, y).solution.t()          # [192][64]
Wt = wt.float().reshape(64, 192).t()                    # [192][64]
for r in range(0, 192, 8):
    d = (Beff[r:r + 8] - Wt[r:r + 8]).abs().max().item()
    if d > 0.01:
        # which true rows match these effective rows?
        m = [int(((Wt - Beff[rr]).abs().max(1).values).argmin()) for rr in range(r, r + 8)]
        md = [round(float((Wt - Beff[rr]).abs().max(1).values.min()), 3) for rr in range(r, r + 8)]
        z = [round(float(Beff[rr].abs().max()), 3) for rr in range(r, r + 8)]
        print("rows", r, "err", round(d, 3), "closest true rows", m, "dist", md, "max|B|", z)
print("done")
