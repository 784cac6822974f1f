"""Per-variant LDS conflict ratio of bench/dgrad_conflict_probe.py's counter pass (dispatches in launch order)."""
import glob
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_summary import load, short  # noqa: E402

path = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
ds = [d for d in load(path) if "conv_fd_v2" in d["name"] or "dgrad_zero" in d["name"]]
names = ["plain", "bstat", "acc", "both"]
for t in range(len(ds) // 40):
    for v, nm in enumerate(names):
        grp = ds[t * 40 + v * 10:t * 40 + (v + 1) * 10]
        conf = sum(d.get("SQ_LDS_BANK_CONFLICT", 0) for d in grp)
        act = sum(d.get("SQ_LDS_IDX_ACTIVE", 0) for d in grp)
        dur = sum(d["dur"] for d in grp) / len(grp) * 1e6
        print("%-40s %-6s conflicts %5.1f %%  %.1f us" % (short(grp[0]["name"]), nm, 100.0 * conf / max(act, 1), dur))
