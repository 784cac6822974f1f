"""Graph-timed BERT-base FFN-out data gradient with the GELU backward on the GEMM core (mm.dgrad with act_pre):
dH [8192 x 3072] = dY [8192 x 768] W2^T * gelu'(pre).  One JSON line (MDTF_PP_PRE_LDS selects the LDS-staged or
direct pre-activation loads of the epilogue; run once per setting)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from bench.gemm_pp_probe import gtime  # noqa: E402
from mdtf.ops import mm  # noqa: E402


def main():
    M, K, Nn = 8192, 3072, 768
    dy = (torch.rand(M, Nn, device="cuda") * 2 - 1).bfloat16()
    w2 = (torch.rand(K, Nn, device="cuda") * 0.1 - 0.05).bfloat16()
    pre = torch.randn(M, K, device="cuda").bfloat16()
    out = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
    plain = gtime(lambda: mm.dgrad(dy, [w2], out=out)) * 1000.0
    act = gtime(lambda: mm.dgrad(dy, [w2], out=out, act_pre=pre, act_bwd=2)) * 1000.0
    x = pre.float()
    s = torch.sigmoid(1.5957691216 * (x + 0.044715 * x ** 3))
    gg = s + 2 * x * s * (1 - s) * 0.7978845608 * (1 + 0.134145 * x ** 2)
    ref = (dy.float() @ w2.float().t()) * gg
    mm.dgrad(dy, [w2], out=out, act_pre=pre, act_bwd=2)
    err = ((out.float() - ref).norm() / ref.norm()).item()
    print(json.dumps({"pre_lds": os.environ.get("MDTF_PP_PRE_LDS", "1"), "plain_us": round(plain, 2),
                      "act_us": round(act, 2), "rel_err": round(err, 5)}), flush=True)


if __name__ == "__main__":
    main()
