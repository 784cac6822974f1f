#!/usr/bin/env python
"""Summarise a rocprofv3 kernel_stats.csv: per-kernel ms per step and category totals."""
import csv
import re
import sys


CATS = [("conv(mdtf)", r"conv_fd|conv_wgrad"), ("gemm(hipBLASLt)", r"Cijk"),
        ("conv(MIOpen)", r"^(naive_conv|igemm|MIOpen|miopen|ck::|gridwise|sp3A|kernel_batched|SubTensor)"),
        ("batchnorm", r"bn_|batchnorm"), ("optimizer", r"adam_kernel|sgd|momentum"),
        ("attention(mdtf)", r"attn_"), ("transformer", r"ln_|softmax|embed"), ("elementwise(torch)", r"at::native"),
        ("mdtf misc", r"bias_act|act_bwd|colsum|reduce_partials|pool|gap_|xent|transpose|lrn")]


def main(path, steps):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    cat = {}
    print("total GPU ms per step: %.3f" % (tot / 1e6 / steps))
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        ms = float(r["TotalDurationNs"]) / 1e6 / steps
        name = r["Name"]
        c = next((c for c, pat in CATS if re.search(pat, name)), "other")
        cat[c] = cat.get(c, 0.0) + ms
    for c, v in sorted(cat.items(), key=lambda t: -t[1]):
        print("  %-20s %7.3f ms" % (c, v))
    print("top kernels:")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
        print("  %7.3f ms %6d %8.1fus  %s" % (float(r["TotalDurationNs"]) / 1e6 / steps, int(r["Calls"]),
                                            float(r["TotalDurationNs"]) / 1e3 / int(r["Calls"]), r["Name"][:90]))


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0)
