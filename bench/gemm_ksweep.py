"""Graph-timed GEMM time vs reduction length K at a fixed output (M x N): separates the per-tile fixed cost
(pipeline fill, epilogue stores, wave tail) from the K loop, for hipBLASLt (torch.mm) and each tile of the
GEMM core (mdtf/csrc/gemm_pp.hip).  One JSON line per (N, engine) with the times and the least-squares fit
t(K) = a + b K over the sweep.

  python bench/gemm_ksweep.py [--M 8192] [--N 768,3072] [--K 64,128,256,512,768,1536,3072]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from bench.gemm_pp_probe import gtime, rnd  # noqa: E402
from mdtf.ops import mm  # noqa: E402


def fit(ks, ts):
    n = len(ks)
    mk, mt = sum(ks) / n, sum(ts) / n
    b = sum((k - mk) * (t - mt) for k, t in zip(ks, ts)) / sum((k - mk) ** 2 for k in ks)
    return mt - b * mk, b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=8192)
    ap.add_argument("--N", default="768,3072")
    ap.add_argument("--K", default="64,128,256,512,768,1536,3072")
    ap.add_argument("--tiles", default="0,1,2,3,4,5")
    a = ap.parse_args()
    ks = [int(k) for k in a.K.split(",")]
    tiles = [int(t) for t in a.tiles.split(",")]
    for Nn in (int(n) for n in a.N.split(",")):
        rows = {"hipblaslt": {}}
        for t in tiles:
            rows["t%d" % t] = {}
        for K in ks:
            x, w = rnd(a.M, K), rnd(K, Nn)
            rows["hipblaslt"][K] = gtime(lambda: torch.mm(x, w)) * 1000.0
            for t in tiles:
                if mm.fwd(x, w, tile=t) is not None:
                    rows["t%d" % t][K] = gtime(lambda: mm.fwd(x, w, tile=t)) * 1000.0
        for eng, d in rows.items():
            if len(d) < 2:
                continue
            kk = sorted(d)
            a0, b0 = fit(kk, [d[k] for k in kk])
            tf = {k: round(2.0 * a.M * Nn * k / (d[k] * 1e-6) / 1e12, 1) for k in kk}
            print(json.dumps({"M": a.M, "N": Nn, "engine": eng, "us": {k: round(d[k], 2) for k in kk},
                              "TFs": tf, "fit_fixed_us": round(a0, 2), "fit_us_per_k64": round(b0 * 64, 3)}),
                  flush=True)


if __name__ == "__main__":
    main()
