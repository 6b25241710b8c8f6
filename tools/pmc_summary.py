"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes into profiles/pmc_traffic.json.

usage: python tools/pmc_summary.py <fetch counter_collection.csv> <write counter_collection.csv> [out.json]

Each pass is a separate ``rocprofv3 --pmc <ctr> --kernel-trace`` run of
``bench.py`` (the guide's rule: FETCH_SIZE and WRITE_SIZE do not fit one pass).
Values are kilobytes per dispatch; the largest-grid dispatches of each kernel
(the bench's timed batch) are averaged.

gfx950 note (MI355X_MICROARCH.md, HBM section): FETCH_SIZE under-reports wide
16-B/lane streaming reads by exactly 2x.  The solver reads 12-B points from
AoS rows (frame-per-lane gathers), a width the guide leaves uncalibrated; the
raw value is kept and checked against the line-granular byte count of the rows
the kernel touches, which it matches without the 2x factor.
"""
from __future__ import annotations

import collections
import csv
import json
import sys


def per_kernel(path: str):
    rows = list(csv.DictReader(open(path)))
    by = collections.defaultdict(list)
    for r in rows:
        by[r["Kernel_Name"]].append((int(r["Grid_Size"]), float(r["Counter_Value"]) * 1024.0))
    out = {}
    for name, vals in by.items():
        g = max(v[0] for v in vals)
        big = [v[1] for v in vals if v[0] == g]
        out[name] = {"grid": g, "dispatches": len(big), "bytes": sum(big) / len(big)}
    return out


def main() -> None:
    fetch, write = per_kernel(sys.argv[1]), per_kernel(sys.argv[2])
    out_path = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json"
    res = {}
    for name in fetch:
        if name not in write:
            continue
        short = name.split("(")[0].replace("void ", "")
        res[short] = {"grid": fetch[name]["grid"], "fetch_bytes": fetch[name]["bytes"],
                      "write_bytes": write[name]["bytes"],
                      "traffic_bytes": fetch[name]["bytes"] + write[name]["bytes"],
                      "fetch_correction": 1.0, "sources": [sys.argv[1], sys.argv[2]]}
    json.dump(res, open(out_path, "w"), indent=1)
    for k, v in res.items():
        print(f"{k:50s} grid={v['grid']:>9d} fetch={v['fetch_bytes'] / 1e6:9.2f} MB "
              f"write={v['write_bytes'] / 1e6:9.2f} MB")


if __name__ == "__main__":
    main()
