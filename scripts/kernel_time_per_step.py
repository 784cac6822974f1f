#!/usr/bin/env python
"""GPU kernel time per training step from a rocprofv3 kernel trace: steps are delimited by a kernel that runs
once per step (regex); reports, over the last N steps, the median kernel-busy time (sum of kernel durations)
and the median span.  usage: kernel_time_per_step.py <run_kernel_trace.csv> <delimiter regex> [N]"""
import csv
import re
import statistics
import sys


def main(path, delim, n=10):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    cut = [i for i, r in enumerate(rows) if re.search(delim, r["Kernel_Name"])]
    steps = [rows[a:b] for a, b in zip(cut[:-1], cut[1:])][-int(n):]
    busy = [sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in s) / 1e6 for s in steps]
    span = [(int(s[-1]["End_Timestamp"]) - int(s[0]["Start_Timestamp"])) / 1e6 for s in steps]
    print("steps %d kernels/step %d busy %.3f ms span %.3f ms" % (len(steps), len(steps[-1]), statistics.median(busy),
                                                                  statistics.median(span)))


if __name__ == "__main__":
    main(*sys.argv[1:])
