#!/usr/bin/env python
"""Per-category GPU time of ONE steady-state training step from a rocprofv3 kernel trace
(steps delimited by the fused optimizer launch).  usage: step_breakdown.py <run_kernel_trace.csv>"""
import collections
import csv
import re
import sys

WS = r"conv_ws_kernel<\d+, \d+, \d+, \d+, \d+, "     # ...<TP, NW, CG, D, KSC, EPI, DIRECT>
CATS = [("conv_fwd", r"conv_fd_v2<\d+, \d+, 0, |conv_fd_kernel<\d+, \d+, 0,|" + WS + r"1,|stem_pack4"),
        ("conv_dgrad", r"conv_fd_v2<\d+, \d+, [12], |conv_fd_kernel<\d+, \d+, [12],|" + WS + r"[234],"),
        ("conv_ws_plain", WS + r"0,"), ("conv_wgrad", r"conv_wgrad|stem_wgrad"),
        ("winograd", r"wino"),
        ("miopen", r"^(naive_conv|igemm|MIOpen|miopen|ck::|gridwise|sp3A|kernel_batched|SubTensor|_ZN2ck)"),
        ("bn_apply", r"bn_apply"), ("bn_dx", r"bn_dx"), ("bn_reduce", r"bn_reduce"), ("bn_finalize", r"bn_finalize"),
        ("optimizer", r"momentum|adam_kernel|sgd_kernel"), ("pool", r"pool"), ("transpose", r"transpose"),
        ("torch", r"at::native"), ("gemm", r"Cijk"), ("rccl", r"nccl|rccl")]


def main(path):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if re.search(r"momentum_kernel|adam_kernel|sgd_kernel", r["Kernel_Name"])]
    ends, prev = [], -10
    for i in idx:
        if i - prev > 5:
            ends.append(i)
        prev = i
    segs = [rows[a + 1:b + 1] for a, b in zip(ends[:-1], ends[1:])]
    segs = [s for s in segs if s]
    spans = [(int(s[-1]["End_Timestamp"]) - int(s[0]["Start_Timestamp"])) / 1e6 for s in segs]
    seg = sorted(zip(spans, range(len(segs))))[len(segs) // 2][1]     # the median-span step
    seg = segs[seg]
    cat, cnt = collections.defaultdict(float), collections.Counter()
    for r in seg:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        c = next((c for c, p in CATS if re.search(p, r["Kernel_Name"])), "other")
        cat[c] += d
        cnt[c] += 1
    span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e6
    print("steps found: %d; median step: %d kernels, span %.2f ms, busy %.2f ms" % (
        len(segs), len(seg), span, sum(cat.values())))
    for c, v in sorted(cat.items(), key=lambda t: -t[1]):
        print("  %-12s %6.2f ms  %4d kernels" % (c, v, cnt[c]))


if __name__ == "__main__":
    main(sys.argv[1])
