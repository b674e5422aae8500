#!/usr/bin/env python3
"""Mean PMC counter per kernel name from rocprofv3 --pmc passes (counter_collection
CSVs found recursively under each directory).  FETCH_SIZE is doubled per the
gfx950 correction (MI355X_MICROARCH.md, HBM section); both are reported in bytes.
usage: pmc_kernel_summary.py DIR [DIR ...]  -> one JSON line per (dir, kernel, counter)"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    for d in sys.argv[1:]:
        acc = defaultdict(list)
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    acc[(row["Kernel_Name"], row["Counter_Name"])].append(float(row["Counter_Value"]))
        for (k, c), v in sorted(acc.items()):
            m = sum(v) / len(v)
            if c not in ("FETCH_SIZE", "WRITE_SIZE"):      # event counts, not KiB
                print(json.dumps({"dir": os.path.basename(d.rstrip("/")), "kernel": k[:120], "counter": c,
                                  "per_dispatch": round(m), "dispatches": len(v)}))
                continue
            m *= 1024.0
            if c == "FETCH_SIZE":
                m *= 2.0
            print(json.dumps({"dir": os.path.basename(d.rstrip("/")), "kernel": k[:120], "counter": c,
                              "bytes_per_dispatch": round(m), "dispatches": len(v)}))


if __name__ == "__main__":
    main()
