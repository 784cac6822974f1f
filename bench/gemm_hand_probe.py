#!/usr/bin/env python
"""Hand-written MFMA GEMM (the v2/v3 implicit-GEMM conv kernels run as a 1x1 convolution) vs hipBLASLt
(torch.mm) on the BERT-base dense shapes: forward y = x W (+ filter transpose) and data gradient dx = dy W^T."""
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from mdtf.ops import conv as C  # noqa: E402
from mdtf.ops import tunable  # noqa: E402

SHAPES = [(8192, 768, 2304), (8192, 768, 768), (8192, 768, 3072), (8192, 3072, 768), (1280, 768, 768)]
TILES = [(128, 128, 2, 2), (128, 128, 3, 2), (128, 64, 3, 2), (64, 128, 3, 2), (256, 128, 2, 3), (256, 256, 2, 3),
         (128, 256, 2, 3), (128, 256, 3, 3), (256, 128, 3, 3), (256, 64, 3, 3)]


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


def main():
    dev = torch.device("cuda")
    tunable.ensure(dev)
    out = []
    for M, K, N in SHAPES:
        x = torch.randn(M, K, device=dev).bfloat16()
        w = (torch.randn(K, N, device=dev) * 0.03).bfloat16()
        dy = torch.randn(M, N, device=dev).bfloat16()
        fl = 2.0 * M * K * N
        t_lib_f = timeit(lambda: torch.mm(x, w))
        t_lib_d = timeit(lambda: torch.mm(dy, w.t()))
        x4 = x.view(1, 1, M, K)
        w4 = w.view(1, 1, K, N)
        best_f = best_d = None
        for bm, bn, st, ver in TILES:
            try:
                tf = timeit(lambda: C.mdtf_fwd(x4, w4, (1, M), (1, 1), (0, 0, 0, 0), (1, 1), bm, bn, None, ver, st))
                if best_f is None or tf < best_f[0]:
                    best_f = (tf, (bm, bn, st, ver))
            except RuntimeError:
                pass
            try:
                td = timeit(lambda: C.mdtf_dgrad(dy.view(1, 1, M, N), w4, (1, 1, M, K), (1, 1), (0, 0, 0, 0), (1, 1),
                                                 bm, bn, ver, st))
                if best_d is None or td < best_d[0]:
                    best_d = (td, (bm, bn, st, ver))
            except RuntimeError:
                pass
        t_tr = timeit(lambda: C.transpose_filter(w4))
        y_ref = torch.mm(x.float(), w.float())
        y = C.mdtf_fwd(x4, w4, (1, M), (1, 1), (0, 0, 0, 0), (1, 1), *best_f[1][:2], None, best_f[1][3], best_f[1][2])
        err = ((y.view(M, N).float() - y_ref).norm() / y_ref.norm()).item()
        rec = {"M": M, "K": K, "N": N, "lib_fwd_ms": round(t_lib_f, 4), "mdtf_fwd_ms": round(best_f[0], 4),
               "fwd_tile": best_f[1], "transpose_ms": round(t_tr, 4), "lib_dgrad_ms": round(t_lib_d, 4),
               "mdtf_dgrad_ms": round(best_d[0], 4), "dgrad_tile": best_d[1],
               "lib_fwd_TFs": round(fl / t_lib_f / 1e9), "mdtf_fwd_TFs": round(fl / best_f[0] / 1e9), "rel_err": err}
        print(json.dumps(rec), flush=True)
        out.append(rec)


if __name__ == "__main__":
    main()
