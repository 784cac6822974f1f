#!/usr/bin/env python
"""GPU kernel time per training step from two rocprofv3 --stats runs of the same benchmark with different
step counts: (total kernel ns of the long run - of the short run) / (step difference).  Build, warm-up and
autotune passes cancel.  usage: kernel_time_diff.py <short_kernel_stats.csv> <S_short> <long_kernel_stats.csv> <S_long>"""
import csv
import sys


def total_ns(path):
    return sum(float(r["TotalDurationNs"]) for r in csv.DictReader(open(path)))


def main(a, sa, b, sb):
    per = (total_ns(b) - total_ns(a)) / (int(sb) - int(sa)) / 1e6
    print("%.3f" % per)


if __name__ == "__main__":
    main(*sys.argv[1:5])
