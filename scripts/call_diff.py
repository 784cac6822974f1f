#!/usr/bin/env python
"""Per-call kernel time difference of two `step_breakdown.py --calls` summaries of the same step (same kernel
issue order, e.g. an env A/B): one line per call whose kernel name contains the filter, plus the summed delta.

usage: call_diff.py <summary_A.txt> <summary_B.txt> [name filter]"""
import re
import sys


def calls(path):
    out, on = [], False
    for line in open(path):
        if line.startswith("calls in issue order"):
            on = True
            continue
        m = re.match(r"\s+([\d.]+)\s+([\d.]+)\s+(.*)", line) if on else None
        if m:
            out.append((float(m.group(2)), m.group(3).strip()))
    return out


def main(a, b, filt=""):
    ca, cb = calls(a), calls(b)
    tot_a = tot_b = 0.0
    for (ta, na), (tb, nb) in zip(ca, cb):
        if filt not in na:
            continue
        tot_a += ta
        tot_b += tb
        tag = "" if na == nb else "   [B: %s]" % nb[:60]
        print("%8.1f %8.1f %+7.1f  %s%s" % (ta, tb, tb - ta, na[:80], tag))
    print("total %.1f -> %.1f us (%+.1f)" % (tot_a, tot_b, tot_b - tot_a))


if __name__ == "__main__":
    main(*sys.argv[1:4])
