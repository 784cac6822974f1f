"""A few launches of each GEMM-core variant (and the hipBLASLt reference) for a rocprofv3 --pmc pass."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mdtf.ops import mm  # noqa: E402


def rnd(*shape):
    return (torch.rand(*shape, device="cuda") * 2 - 1).to(torch.bfloat16)


def main(reps=5):
    cases = []
    for (M, Nn, K, tile) in ((8192, 8192, 8192, 0), (8192, 768, 768, 5), (8192, 3072, 768, 4)):
        x, w, wT = rnd(M, K), rnd(K, Nn), rnd(Nn, K)
        cases.append(lambda x=x, w=w, tile=tile: mm.fwd(x, w, tile=tile))
        cases.append(lambda x=x, wT=wT, tile=tile: mm.dgrad(x, wT, tile=tile))
        cases.append(lambda x=x, w=w: torch.mm(x, w))
    for (M, Nn, K, tile, sp) in ((768, 2304, 8192, 3, 2), (768, 3072, 8192, 3, 1)):
        xa, dya = rnd(K, M), rnd(K, Nn)
        gw = torch.zeros(M, Nn, device="cuda")
        cases.append(lambda xa=xa, dya=dya, gw=gw, tile=tile, sp=sp: mm.wgrad_into(gw, xa, dya, tile=tile, splits=sp))
    for c in cases:
        for _ in range(reps):
            c()
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
