"""Graph-timed BERT-base weight gradients (T = 8192 tokens) on csrc/gemm_wg.hip: the tiles x splits grid vs
stream-K at several worker counts, alternating in one process.  One JSON line per (shape, arm, round) and a
median summary."""
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from bench.gemm_pp_probe import gtime  # noqa: E402
from mdtf.ops import mm  # noqa: E402

SHAPES = [(768, 2304), (768, 3072), (3072, 768)]


def main():
    T = 8192
    dev = "cuda"
    print(json.dumps({"cus": torch.cuda.get_device_properties(0).multi_processor_count}), flush=True)
    res = {}
    for K, N in SHAPES:
        x = (torch.rand(T, K, device=dev) * 2 - 1).bfloat16()
        dy = (torch.rand(T, N, device=dev) * 2 - 1).bfloat16()
        g = torch.zeros(K, N, device=dev)
        bm, st, sp = mm.wg_pick(K, N, T)
        arms = {"classic": sp}
        for gw in [int(v) for v in os.environ.get("SK_G", "216,256,512,128").split(",")]:
            arms["sk%d" % gw] = -gw
        key = "%dx%d" % (K, N)
        res[key] = {a: [] for a in arms}
        for rnd in range(3):
            for arm, splits in arms.items():
                mm.WG_SK = False
                fn = lambda s=splits: mm.wg_into([g], x, dy, bm=bm, stages=st, splits=s)  # noqa: E731
                t = gtime(fn) * 1000.0
                res[key][arm].append(t)
                print(json.dumps({"shape": key, "arm": arm, "splits": splits, "round": rnd, "us": round(t, 2)}),
                      flush=True)
    print(json.dumps({"summary": {k: {a: round(statistics.median(v), 2) for a, v in d.items()}
                                  for k, d in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
