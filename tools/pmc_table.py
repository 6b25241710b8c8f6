"""Per-kernel table of a rocprofv3 PMC directory tree (one subdirectory per pass): every counter summed over a
dispatch's rows, averaged over the dispatches at the kernel's largest grid, plus the kernel-trace average time.
usage: python tools/pmc_table.py <dir> [kernel-substring ...]"""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import sys


def main(d, pats):
    acc = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    grid = {}
    for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if pats and not any(p in name for p in pats):
                continue
            g = int(r["Grid_Size"])
            key = (name, g)
            acc[key][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
            grid[name] = max(grid.get(name, 0), g)
    out = {}
    for (name, g), cs in acc.items():
        if g != grid[name]:
            continue
        out[name] = {"grid": g, **{c: sum(v.values()) / len(v) for c, v in cs.items()}}
    for f in glob.glob(os.path.join(d, "trace", "*kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Name"].split("(")[0].replace("void ", "")
            if name in out:
                out[name]["avg_ns"] = float(r["AverageNs"])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
