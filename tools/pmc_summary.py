"""Summarise a round's rocprofv3 PMC passes into one JSON that bench.py reads (profiles/pmc_<tag>.json).

usage: python tools/pmc_summary.py <pmc dir> [out.json]

<pmc dir> is what tools/profile_round.sh writes on the GPU box:
  fetch/ write/          FETCH_SIZE / WRITE_SIZE passes of `bench.py --steps 10` (one counter family per pass)
  sq/                    SQ_WAVES + VALU instruction counters of the same command
  notab_fetch/           FETCH_SIZE of the RTG_EXP_NO_TABLE build (the angle table's share of the fetch)
  calib_fetch/ calib_write/  FETCH_SIZE / WRITE_SIZE of tools/fetch_calib (known-byte micro-kernels)
  calib.json             the byte counts tools/fetch_calib printed
Counters are summed over a dispatch's rows and averaged over the dispatches at the kernel's largest grid.

FETCH_SIZE calibration (MI355X_MICROARCH.md, HBM section: only 16 B/lane streaming reads are calibrated, where the
counter reports exactly 1/2, i.e. 128-byte requests tallied at 64 B).  Measured here: k_stream16 known/counter =
2.00; k_gather<63,21> -- every byte of the AoS rows read once with the solver's 12-byte frame-per-lane loads --
1.86, i.e. the same 2x unit with ~8 % of its lines requested twice (L2 evictions between the 21 point loads of a
row; that kernel's known byte count is a lower bound on its traffic).  So FETCH_SIZE counts 128-byte line requests
at 64 B for the gather shape too, and the solver's calibrated fetch = raw x the k_stream16 factor; the gather
kernels' ratios are kept in the JSON as the evidence.  Infinity-Cache (MALL) hits are counted, not excluded.
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import statistics
import sys


def load(d: str):
    """kernel name -> {counter: mean per-dispatch value at the largest grid}, and that grid."""
    acc = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    grid = {}
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            g = int(r["Grid_Size"])
            if g < grid.get(name, -1):
                continue
            if g > grid.get(name, -1):
                grid[name] = g
                acc[name].clear()
            acc[name][r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {}
    for name, per in acc.items():
        names = {c for v in per.values() for c in v}
        out[name] = {"grid": grid[name], "dispatches": len(per),
                     **{c: statistics.mean(v[c] for v in per.values() if c in v) for c in names}}
    return out


SOLVERS = ("rtg::k_solve_sides<0, true, true>",    # SoA inputs (the bench headline)
           "rtg::k_solve_sides<0, true, false>")   # AoS rows (the reference's layout, secondary line)
VALU_PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9    # CUs x SIMDs x lanes/cycle x clock (fp32 FMA-issue rate)


def solver_record(SOLVER, fetch, write, sq, nt, factor, kb):
    """Calibrated traffic and the SQ instruction mix of one solver kernel."""
    rec = {"kernel": SOLVER, "grid": fetch[SOLVER]["grid"], "fetch_size_raw": fetch[SOLVER]["FETCH_SIZE"] * kb,
           "write_bytes": write[SOLVER]["WRITE_SIZE"] * kb, "fetch_correction": factor,
           "fetch_correction_source": "tools/fetch_calib.hip k_stream16 (counter unit: 128-B requests at 64 B); "
                                      "k_gather<63, 21> corroborates for the 12-byte gather shape"}
    rec["fetch_bytes"] = rec["fetch_size_raw"] * factor
    rec["traffic_bytes"] = rec["fetch_bytes"] + rec["write_bytes"]
    if SOLVER in nt:
        rec["fetch_bytes_no_angle_table"] = nt[SOLVER]["FETCH_SIZE"] * kb * factor
        rec["angle_table_fetch_bytes"] = rec["fetch_bytes"] - rec["fetch_bytes_no_angle_table"]
    s = sq.get(SOLVER, {})
    if "SQ_INSTS_VALU" in s:
        rec["valu_insts"] = s["SQ_INSTS_VALU"]
        rec["waves"] = s.get("SQ_WAVES")
        # issue weights: f64 add/mul/fma at half rate, f64 transcendentals at an eighth, f32 ones at a quarter
        w64 = sum(s.get(f"SQ_INSTS_VALU_{k}_F64", 0.0) for k in ("ADD", "MUL", "FMA"))
        rec["valu_issue_weighted"] = (s["SQ_INSTS_VALU"] + w64 + 7 * s.get("SQ_INSTS_VALU_TRANS_F64", 0.0) +
                                      3 * s.get("SQ_INSTS_VALU_TRANS_F32", 0.0))
        rec.update({k: v for k, v in s.items() if k.startswith("SQ_")})
    return rec


def main() -> None:
    d = sys.argv[1]
    out_path = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_r03.json"
    kb = 1024.0   # FETCH_SIZE / WRITE_SIZE are in KB
    fetch, write, sq = load(os.path.join(d, "fetch")), load(os.path.join(d, "write")), load(os.path.join(d, "sq"))
    res = {"sources": sorted(os.path.relpath(p, d) for p in glob.glob(os.path.join(d, "*", "*counter_collection.csv")))}
    calib = {}
    cj = os.path.join(d, "calib.json")
    if os.path.exists(cj):
        known = json.load(open(cj))
        cf, cw = load(os.path.join(d, "calib_fetch")), load(os.path.join(d, "calib_write"))
        for k in ("k_stream16", "k_gather<63, 21>", "k_gather<63, 10>", "k_gather<60, 11>"):
            full = next((n for n in cf if n.endswith(k)), None)
            if full is None:
                continue
            f = cf[full]["FETCH_SIZE"] * kb
            calib[k] = {"fetch_size_bytes": f, "known_bytes": known[k]["bytes"],
                        "known_line_bytes": known[k].get("line_bytes"), "known_over_counter": known[k]["bytes"] / f}
            w = next((n for n in cw if n.endswith(k)), None)
            if w is not None:
                calib[k]["write_size_bytes"] = cw[w]["WRITE_SIZE"] * kb
                calib[k]["known_write_bytes"] = known[k]["write_bytes"]
        res["calibration"] = calib
    factor = calib.get("k_stream16", {}).get("known_over_counter", 2.0)
    nt = load(os.path.join(d, "notab_fetch"))
    for SOLVER in SOLVERS:
        if SOLVER not in fetch:
            continue
        res[SOLVER] = rec = solver_record(SOLVER, fetch, write, sq, nt, factor, kb)
        print(SOLVER)
        print(json.dumps({k: (round(v / 1e6, 2) if isinstance(v, float) and v > 1e5 else v) for k, v in rec.items()},
                         indent=1))
    json.dump(res, open(out_path, "w"), indent=1)
    for k, v in calib.items():
        print(f"calib {k:18s} counter {v['fetch_size_bytes'] / 1e6:9.2f} MB  known {v['known_bytes'] / 1e6:9.2f} MB  "
              f"known/counter {v['known_over_counter']:.3f}")


if __name__ == "__main__":
    main()
