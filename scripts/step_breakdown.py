#!/usr/bin/env python
"""Per-category and per-kernel GPU time of ONE steady-state training step from a rocprofv3 kernel trace
(steps delimited by the fused optimizer launch).

usage: step_breakdown.py <run_kernel_trace.csv | rocprofv3 output dir> [--calls]

Every number printed comes from the same median-span step, so the category sum equals the "busy" total and
the top-kernel list sums to it too (no mixing of whole-trace stats with per-step numbers)."""
import collections
import csv
import glob
import os
import re
import sys

WS = r"conv_ws_kernel<\d+, \d+, \d+, \d+, \d+, "     # ...<TP, NW, CG, D, KSC, EPI, DIRECT>
CATS = [("conv_fwd", r"conv_fd_v2<\d+, \d+, 0, |conv_fd_kernel<\d+, \d+, 0,|conv_pp|" + WS + r"1,|stem_pack4|stem_conv_rows"),
        ("conv_dgrad", r"conv_fd_v2<\d+, \d+, [12], |conv_fd_kernel<\d+, \d+, [12],|dgrad_zero_classes|" + WS + r"[234],"),
        ("conv_ws_plain", WS + r"0,"), ("conv_wgrad", r"conv_wgrad|stem_wgrad"),
        ("winograd", r"wino"),
        ("miopen", r"^(naive_conv|igemm|MIOpen|miopen|ck::|gridwise|sp3A|kernel_batched|SubTensor|_ZN2ck)"),
        ("bn_apply", r"bn_apply|bn_relu_maxpool"), ("bn_dx", r"bn_dx|maxpool_bn"), ("bn_reduce", r"bn_reduce"),
        ("bn_finalize", r"bn_finalize"),
        ("optimizer", r"momentum|adam_kernel|sgd_kernel"), ("pool", r"pool"), ("transpose", r"transpose"),
        ("attention", r"attn"), ("gemm_hand", r"gemm_pp|gemm_wg|dense_"), ("layernorm", r"ln_|layernorm"),
        ("torch", r"at::native"), ("rocclr", r"rocclr"), ("gemm_lib", r"Cijk"), ("rccl", r"nccl|rccl")]


def _csv(path):
    if os.path.isdir(path):
        c = sorted(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True))
        if not c:
            raise SystemExit("no *kernel_trace.csv under %s" % path)
        return c[0]
    return path


def _short(name, n=90):
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"\(.*$", "", name) if "<" not in name.split("(")[0] else re.sub(r"\)\(.*$", ")", name)
    return name[:n]


def main(path, calls=False):
    rows = sorted(csv.DictReader(open(_csv(path))), key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if re.search(r"momentum_kernel|adam_kernel|sgd_kernel", r["Kernel_Name"])]
    ends, prev = [], -10
    for i in idx:
        if i - prev > 5:
            ends.append(i)
        prev = i
    segs = [rows[a + 1:b + 1] for a, b in zip(ends[:-1], ends[1:])]
    segs = [s for s in segs if s]
    if not segs:
        raise SystemExit("no complete step between two optimizer launches")
    spans = [(int(s[-1]["End_Timestamp"]) - int(s[0]["Start_Timestamp"])) / 1e6 for s in segs]
    seg = segs[sorted(zip(spans, range(len(segs))))[len(segs) // 2][1]]     # the median-span step
    cat, cnt = collections.defaultdict(float), collections.Counter()
    per_k, per_n = collections.defaultdict(float), collections.Counter()
    for r in seg:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        c = next((c for c, p in CATS if re.search(p, r["Kernel_Name"])), "other")
        cat[c] += d
        cnt[c] += 1
        per_k[r["Kernel_Name"]] += d
        per_n[r["Kernel_Name"]] += 1
    span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1e6
    busy = sum(cat.values())
    print("steps found: %d; median step: %d kernels, span %.2f ms, busy %.2f ms (sum of kernel durations; "
          "> span where kernels overlap)" % (len(segs), len(seg), span, busy))
    for c, v in sorted(cat.items(), key=lambda t: -t[1]):
        print("  %-13s %6.2f ms  %4d kernels" % (c, v, cnt[c]))
    print("top kernels of that step (ms, calls, us/call):")
    for k, v in sorted(per_k.items(), key=lambda t: -t[1])[:40]:
        print("  %7.3f ms %4d %8.1f us  %s" % (v, per_n[k], 1000 * v / per_n[k], _short(k)))
    if calls:
        print("calls in issue order (us):")
        t0 = int(seg[0]["Start_Timestamp"])
        for r in seg:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            print("  %9.1f %8.1f  %s" % ((int(r["Start_Timestamp"]) - t0) / 1e3, d, _short(r["Kernel_Name"], 110)))


if __name__ == "__main__":
    main(sys.argv[1], "--calls" in sys.argv)
