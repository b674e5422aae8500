#!/usr/bin/env python3
"""pmc_db.py -- per-dispatch counter totals from a rocprofv3 --pmc database
(the rocpd SQLite file rocprofv3 writes by default: counters_collection view).

usage: pmc_db.py DB [--match SUBSTR] [--min VALUE]
Prints, per kernel dispatch: short kernel name, grid, scratch, VGPRs and the
sum of each counter over its instances (XCDs / SEs).  FETCH_SIZE and
WRITE_SIZE are in KiB (the guide's gfx950 notes apply to their reading)."""
import argparse
import collections
import re
import sqlite3


def short(name):
    name = re.sub(r"\(.*", "", name)
    return name[-90:]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--match", default="")
    ap.add_argument("--min", type=float, default=0.0)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = con.execute("select dispatch_id, kernel_name, grid_size, scratch_size, vgpr_count, counter_name, value "
                       "from counters_collection order by dispatch_id")
    agg = collections.OrderedDict()
    for d, k, g, sc, vg, c, v in rows:
        if a.match and a.match not in k:
            continue
        e = agg.setdefault(d, {"k": short(k), "g": g, "sc": sc, "vg": vg, "c": collections.OrderedDict()})
        e["c"][c] = e["c"].get(c, 0.0) + float(v)
    for d, e in agg.items():
        if max(e["c"].values(), default=0) < a.min:
            continue
        cs = "  ".join(f"{c} {v:.6g}" for c, v in e["c"].items())
        print(f"{d:>5} {e['k']:<90} grid {e['g']:>10} scratch {e['sc']:>4} vgpr {e['vg']:>3}  {cs}")


if __name__ == "__main__":
    main()
