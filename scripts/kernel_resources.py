#!/usr/bin/env python
"""Per-kernel VGPR / spill / occupancy table from `hipcc -Rpass-analysis=kernel-resource-usage` output.

    hipcc ... -c src.hip -Rpass-analysis=kernel-resource-usage 2>&1 | python scripts/kernel_resources.py
"""
import re
import subprocess
import sys

rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    if cur is None:
        continue
    for key, pat in (("vgpr", r"VGPRs: (\d+)"), ("agpr", r"AGPRs: (\d+)"), ("vspill", r"VGPRs Spill: (\d+)"),
                     ("sspill", r"SGPRs Spill: (\d+)"), ("occ", r"Occupancy \[waves/SIMD\]: (\d+)"),
                     ("lds", r"LDS Size \[bytes/block\]: (\d+)")):
        m = re.search(pat, line)
        if m and key not in cur:
            cur[key] = int(m.group(1))
names = [r["name"] for r in rows]
try:
    dem = subprocess.run(["/opt/rocm/llvm/bin/llvm-cxxfilt"], input="\n".join(names), capture_output=True,
                         text=True).stdout.splitlines()
except Exception:
    dem = names
for r, d in zip(rows, dem):
    d = re.sub(r"\(anonymous namespace\)::", "", d).replace("WsArgs", "")
    print("%-60s vgpr %3s agpr %3s vspill %3s sspill %3s occ %s" % (d[:60], r.get("vgpr"), r.get("agpr"),
                                                                    r.get("vspill"), r.get("sspill"), r.get("occ")))
