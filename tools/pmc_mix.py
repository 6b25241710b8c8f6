"""Per-wave instruction mix of one kernel from tools/pmc_passes.sh output.

    python tools/pmc_mix.py gpurun_out/pmc_<tag>_* [--kernel solve_sides] [--grid 524288]

Counters are summed over a dispatch's rows (XCDs / SEs), averaged over the
dispatches of the kernel at that grid size, and divided by SQ_WAVES (taken from
the `sq` pass).  Prints JSON.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import statistics


def load(dirs, kernel, grid):
    per = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "*_counter_collection.csv")):
            acc = collections.defaultdict(lambda: collections.defaultdict(float))
            for r in csv.DictReader(open(f)):
                if kernel in r["Kernel_Name"] and (grid is None or int(r["Grid_Size"]) == grid):
                    acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
            names = {n for v in acc.values() for n in v}
            for n in names:
                per[n] = statistics.mean(v[n] for v in acc.values() if n in v)
    return per


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="solve_sides")
    ap.add_argument("--grid", type=int, default=524288)
    a = ap.parse_args()
    c = load(a.dirs, a.kernel, a.grid)
    waves = c.get("SQ_WAVES")
    out = {"kernel": a.kernel, "grid": a.grid, "totals": c}
    if waves:
        out["per_wave"] = {k: v / waves for k, v in c.items() if k.startswith("SQ_INSTS")}
        f64 = sum(c.get(f"SQ_INSTS_VALU_{k}_F64", 0.0) for k in ("ADD", "MUL", "FMA", "TRANS"))
        f32 = sum(c.get(f"SQ_INSTS_VALU_{k}_F32", 0.0) for k in ("ADD", "MUL", "FMA", "TRANS"))
        if "SQ_INSTS_VALU" in c:
            out["valu_share"] = {"f64": f64 / c["SQ_INSTS_VALU"], "f32": f32 / c["SQ_INSTS_VALU"]}
        if "SQ_WAVE_CYCLES" in c:
            wc = c["SQ_WAVE_CYCLES"]
            out["wave_cycle_split"] = {k: c[k] / wc for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY")
                                       if k in c}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
