#!/usr/bin/env python
"""Merge fresh per-pass autotune tables (bench/conv_autotune.py --out ...) into a candidate conv table.

    python bench/merge_conv_tables.py --base mdtf/ops/conv_table.json --out gpurun_out/conv_table_cand.json \
        --tag slab=gpurun_out/conv_table_wgrad_slab.json --tag atom=gpurun_out/conv_table_wgrad_atom.json

Every ``--tag name=path`` table was measured in one process on one device; for each key present in any of them
the fastest entry wins (``slab=`` entries are marked ``"slab": 1``, others ``"slab": 0`` for the weight-gradient
launcher).  Keys only in the base table are kept.  The candidate is meant for an in-step A/B
(``MDTF_CONV_TABLE=<out>``), not to be trusted from isolated timings alone.
"""
import argparse
import json


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--base", required=True)
    p.add_argument("--out", required=True)
    p.add_argument("--tag", action="append", default=[])
    p.add_argument("--passes", default="wgrad")
    a = p.parse_args()
    base = json.load(open(a.base))
    best = {}
    for t in a.tag:
        name, path = t.split("=", 1)
        for k, ent in json.load(open(path)).items():
            if k.split(":")[0] not in a.passes.split(",") or ent.get("backend") != "mdtf" or "ms" not in ent:
                continue
            e = dict(ent)
            if k.startswith("wgrad:"):
                e["slab"] = 1 if name == "slab" else 0
            if k not in best or e["ms"] < best[k]["ms"]:
                best[k] = e
    changed = 0
    for k, e in sorted(best.items()):
        old = base.get(k)
        same = old is not None and all(old.get(f) == e.get(f)
                                       for f in ("bm", "bn", "splits", "ver", "stages", "ws", "tile"))
        if not same or old.get("slab", 0) != e.get("slab", 0):
            changed += 1
            print("%-45s %s -> %s" % (k, {f: (old or {}).get(f) for f in ("bm", "bn", "splits", "stages", "ver", "ws",
                                                                        "tile", "ms")},
                                      {f: e.get(f) for f in ("bm", "bn", "splits", "stages", "ver", "ws", "tile", "slab",
                                                             "ms")}))
        base[k] = e
    json.dump(base, open(a.out, "w"), indent=1, sort_keys=True)
    print("changed %d of %d measured keys -> %s" % (changed, len(best), a.out))


if __name__ == "__main__":
    main()
