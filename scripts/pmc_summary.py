#!/usr/bin/env python
"""Summarise the rocprofv3 --pmc passes of scripts/gpu_pmc.sh per kernel.

usage: pmc_summary.py <dir prefix, e.g. gpurun_out/pmc1> [top N] [--last-step]

--last-step: only the dispatches of the last training step (from the end of the second-to-last optimizer
launch group to the end of the last one), so model setup, warmup and graph capture do not count.

Per kernel (aggregated over its dispatches in the profiled steps):
  time      summed dispatch time (serialised by the counter collection)
  TF/s      SQ_INSTS_VALU_MFMA_MOPS_BF16 x 512 FLOP / time
  MFMA %    SQ_VALU_MFMA_BUSY_CYCLES / (time x 2.4 GHz x 1024 SIMDs)
  LDS conf  SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles per LDS-array cycle)
  HBM GB/s  (FETCH_SIZE + WRITE_SIZE) KiB / time
  L2 hit    TCC_HIT / (TCC_HIT + TCC_MISS)
--roofline: two more columns per kernel -- the roofline time max(FLOP / 2.5 PF dense bf16, HBM bytes / 6.3 TB/s
  measured copy rate) and that floor as a % of the measured time.  HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE
  (MI355X_MICROARCH.md: FETCH_SIZE reports half the bytes of wide coalesced streaming reads; narrower or L2-resident
  re-reads make this an over-estimate of the floor, i.e. the % an upper bound).
"""
import collections
import csv
import os
import re
import sys

CLOCK = 2.4e9
SIMDS = 1024


OPT = ("adam_kernel", "momentum_kernel", "sgd_kernel", "apply_multi_kernel")


def last_step(ds):
    """Dispatches of the last step: after the second-to-last optimizer group, through the last one."""
    idx = [i for i, d in enumerate(ds) if any(o in d["name"] for o in OPT)]
    groups = []
    for i in idx:
        if groups and i - groups[-1][-1] <= 16:
            groups[-1].append(i)
        else:
            groups.append([i])
    if len(groups) < 2:
        return ds
    return ds[groups[-2][-1] + 1:groups[-1][-1] + 1]


def load(path, step_only=False):
    per = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        d = per.setdefault(int(r["Dispatch_Id"]), {"name": r["Kernel_Name"],
                                                   "dur": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9})
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    ds = [per[k] for k in sorted(per)]
    return last_step(ds) if step_only else ds


def short(name):
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = re.sub(r"\(\(ConvArgs\)\)|\(ConvArgs\)", "", n)
    n = n.replace("void ", "")
    return n[:70]


PEAK_FLOPS = 2.5e15
HBM_BPS = 6.3e12


def main(prefix, top, step_only=False, roofline=False):
    # each pass is its own run: aggregate per kernel name within a pass, then join the passes by name
    aggs = []
    for i in (1, 2, 3):
        agg = collections.defaultdict(lambda: collections.defaultdict(float))
        path = "%s_p%d/run_counter_collection.csv" % (prefix, i)
        if i > 1 and not os.path.exists(path):      # SQ-only runs: one pass
            aggs.append(agg)
            continue
        for d in load(path, step_only):
            a = agg[short(d["name"])]
            a["calls"] += 1
            a["dur"] += d["dur"]
            for k, v in d.items():
                if k not in ("name", "dur"):
                    a[k] += v
        aggs.append(agg)
    a1, a2, a3 = aggs
    rows = sorted(a1.items(), key=lambda t: -t[1]["dur"])
    tot = sum(a["dur"] for _, a in rows)
    if roofline:
        print("| kernel | calls | ms | TF/s | MFMA busy % | LDS bank-conflict % | HBM GB/s (rd+wr) | L2 hit % "
              "| roofline ms (bound) | % of roofline |")
        print("|---|---|---|---|---|---|---|---|---|---|")
    else:
        print("| kernel | calls | ms | TF/s | MFMA busy % | LDS bank-conflict % | HBM GB/s (rd+wr) | L2 hit % |")
        print("|---|---|---|---|---|---|---|---|")
    floor_tot = 0.0
    for name, a in rows[:top]:
        b, c = a2.get(name, {}), a3.get(name, {})
        dur = a["dur"]
        tf = a["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512 / dur / 1e12 if dur else 0
        mf = 100.0 * a["SQ_VALU_MFMA_BUSY_CYCLES"] / (dur * CLOCK * SIMDS) if dur else 0
        lds = 100.0 * a["SQ_LDS_BANK_CONFLICT"] / a["SQ_LDS_IDX_ACTIVE"] if a["SQ_LDS_IDX_ACTIVE"] else 0
        rd = b.get("FETCH_SIZE", 0) * 1024 / b["dur"] / 1e9 if b.get("dur") else 0
        wr = c.get("WRITE_SIZE", 0) * 1024 / c["dur"] / 1e9 if c.get("dur") else 0
        hit = c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0)
        hit = 100.0 * c.get("TCC_HIT_sum", 0) / hit if hit else 0
        line = "| `%s` | %d | %.3f | %.0f | %.1f | %.1f | %.0f + %.0f | %.0f |" % (
            name, a["calls"], dur * 1e3, tf, mf, lds, rd, wr, hit)
        if roofline:
            flops = a["SQ_INSTS_VALU_MFMA_MOPS_BF16"] * 512
            hbm = 2 * b.get("FETCH_SIZE", 0) * 1024 + c.get("WRITE_SIZE", 0) * 1024
            t_mf, t_hbm = flops / PEAK_FLOPS, hbm / HBM_BPS
            floor = max(t_mf, t_hbm)
            floor_tot += floor
            line += " %.3f (%s) | %.0f |" % (floor * 1e3, "MFMA" if t_mf > t_hbm else "HBM",
                                             100.0 * floor / dur if dur else 0)
        print(line)
    print("\nprofiled dispatches (pass 1%s): %d, total serialized kernel time %.2f ms" % (
        ", last step only" if step_only else "", sum(a["calls"] for _, a in rows), tot * 1e3))
    if roofline:
        shown = sum(a["dur"] for _, a in rows[:top])
        print("roofline floor of the %d kernels shown: %.2f ms of their %.2f ms (%.0f %%)" % (
            min(top, len(rows)), floor_tot * 1e3, shown * 1e3, 100.0 * floor_tot / shown if shown else 0))


if __name__ == "__main__":
    pos = [v for v in sys.argv[1:] if not v.startswith("--")]
    main(pos[0], int(pos[1]) if len(pos) > 1 else 40, "--last-step" in sys.argv, "--roofline" in sys.argv)
