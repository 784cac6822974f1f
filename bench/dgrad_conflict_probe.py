"""LDS bank conflicts of the 4-wave 64 x 128 data-gradient tile by epilogue variant (run under rocprofv3 --pmc
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --kernel-trace): the ResNet-50 stage-3 conv1 data gradient (14 x 14,
1024 <- 256 channels, batch 256) launched 10 times each (the last 9 event-timed) as plain / + BN-backward statistics / + pending masked
accumulate / both, in that order, so the dispatch index tells the variant.  The step runs it with both
(`pmc_resnet50_r5g_counters.md`: 8.8 % conflicts); the 8-wave 256 x 256 tiles show 0-1 %."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from mdtf.ops import conv as C  # noqa: E402
import conv_autotune as T  # noqa: E402


def main():
    n, h, w, c, co = 256, 14, 14, 1024, 256
    x = torch.randn(n, h, w, c, device="cuda").bfloat16()
    wt = (torch.randn(1, 1, c, co, device="cuda") * 0.05).bfloat16()
    dy = torch.randn(n, h, w, co, device="cuda").bfloat16()
    M = n * h * w
    mask = torch.full((M * c // 8,), 0x55, dtype=torch.uint8, device="cuda")
    g = torch.randn_like(x)
    out = torch.empty_like(x)
    tiles = [(64, 128, 2, 2), (256, 256, 2, 3)]
    for bm, bn, st, ver in tiles:
        ss = T._stats(c, bm, M)
        variants = [
            ("plain", {}),
            ("bstat", {"bn_stats": (x, mask, ss[0], ss[1], ss[0].shape[0])}),
            ("acc", {"acc_src": (g, mask)}),
            ("both", {"bn_stats": (x, mask, ss[0], ss[1], ss[0].shape[0]), "acc_src": (g, mask)}),
        ]
        for name, kw in variants:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            C.mdtf_dgrad(dy, wt, x.shape, (1, 1), (0, 0, 0, 0), (1, 1), bm, bn, ver, st, out=out, **kw)
            e0.record()
            for _ in range(9):
                C.mdtf_dgrad(dy, wt, x.shape, (1, 1), (0, 0, 0, 0), (1, 1), bm, bn, ver, st, out=out, **kw)
            e1.record()
            torch.cuda.synchronize()
            print("tile %dx%d %-5s %.1f us" % (bm, bn, name, e0.elapsed_time(e1) / 9 * 1000), flush=True)


if __name__ == "__main__":
    main()
