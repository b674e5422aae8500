#!/usr/bin/env python3
"""Per-launch HBM traffic of a kernel from rocprofv3 PMC passes.

usage: pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv>
                      <kernel-substring> <key> [out.json]

FETCH_SIZE and WRITE_SIZE are collected in SEPARATE rocprofv3 --pmc passes
(they do not fit one TCC pass on gfx950).  Both are in KiB.  Per
MI355X_MICROARCH.md (HBM section) FETCH_SIZE reports exactly half of the
bytes of a wide coalesced (16 B/lane) streaming read on gfx950, so it is
doubled; WRITE_SIZE is exact for 16 B/lane streaming stores.  The result
(mean over the matching dispatches) is merged into profiles/pmc_traffic.json
under `key`, which bench.py reads for roofline.traffic.
"""
import csv
import json
import os
import sys


def mean_counter(path, kernel_sub, name):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel_sub in row["Kernel_Name"] and row["Counter_Name"] == name:
                vals.append(float(row["Counter_Value"]))
    if not vals:
        raise SystemExit(f"no {name} rows for {kernel_sub!r} in {path}")
    return sum(vals) / len(vals), len(vals)


def main():
    fetch_csv, write_csv, sub, key = sys.argv[1:5]
    out = sys.argv[5] if len(sys.argv) > 5 else os.path.join(os.path.dirname(__file__), "..", "profiles",
                                                                 "pmc_traffic.json")
    fk, nf = mean_counter(fetch_csv, sub, "FETCH_SIZE")
    wk, nw = mean_counter(write_csv, sub, "WRITE_SIZE")
    rd = fk * 1024 * 2.0
    wr = wk * 1024
    try:
        with open(out) as f:
            d = json.load(f)
    except (OSError, ValueError):
        d = {}
    d[key] = {"kernel_match": sub, "fetch_size_kib_raw": fk, "write_size_kib": wk,
              "read_bytes_corrected": rd, "write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
              "dispatches": [nf, nw],
              "correction": "FETCH_SIZE x2 (gfx950 16B/lane streaming reads), WRITE_SIZE x1"}
    with open(out, "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)
    print(json.dumps(d[key]))


if __name__ == "__main__":
    main()
