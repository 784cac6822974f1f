"""A few launches of weight-gradient kernel configs on BERT-base FFN-in (768 x 3072 over 8192 tokens) for a
rocprofv3 --pmc pass (scripts/gpu.sh py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from mdtf.ops import mm  # noqa: E402


def rnd(*shape):
    return (torch.rand(*shape, device="cuda") * 2 - 1).to(torch.bfloat16)


def main(reps=3):
    x, dy = rnd(8192, 768), rnd(8192, 3072)
    g = torch.zeros(768, 3072, device="cuda")
    for (bm, st, sp) in ((256, 2, 1), (256, 2, 3), (128, 2, 1), (128, 2, 3), (256, 3, 3)):
        for _ in range(reps):
            mm.wg_into([g], x, dy, bm=bm, stages=st, splits=sp)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
