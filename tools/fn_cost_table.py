"""Per-call instruction cost of each tools/fn_cost.hip kernel from its rocprofv3 PMC passes (one call per lane, so a
wave's count is a call's count): every counter per wave, minus the `empty` kernel.
usage: python tools/fn_cost_table.py <pmc dir (one subdirectory per pass)> [out.json]"""
from __future__ import annotations

import collections
import csv
import glob
import json
import os
import re
import sys

NAMES = ["empty", "qexp_component", "cr_acos", "cr_sincos", "f_atan2f", "normalize_angle", "radians_between",
         "qfrom_angle_axis", "qnormalize", "qfrom_rotmat", "cal_joint_quat<3>", "cal_joint_quat<5>", "scipy_as_euler",
         "quat_in_xyz_axis", "shoulder_pr", "elbow_py", "qrotate", "f32 div", "exp_dof (table)", "qmul_norm",
         "hand_x_mean", "cr_sqrt", "sqrt_clamp_rcp", "rcp64+mulr_q", "quat_in_xyz_intrinsic",
         "la_gesdd3 (5-pt A)", "la_lartg", "la_lasv2", "la_larfg<2>"]
# issue cycles of a wave64 instruction relative to a plain f32 op (f64 add/mul/fma x2, f64
# transcendentals x8, f32 transcendentals x4)
WEIGHT = {"SQ_INSTS_VALU_ADD_F64": 1, "SQ_INSTS_VALU_MUL_F64": 1, "SQ_INSTS_VALU_FMA_F64": 1,
          "SQ_INSTS_VALU_TRANS_F64": 7, "SQ_INSTS_VALU_TRANS_F32": 3}


def main(d, out=None):
    acc = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for f in glob.glob(os.path.join(d, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            m = re.search(r"kcost<(\d+)>", r["Kernel_Name"])
            if m:
                # one pass per file: a dispatch id repeats across passes
                acc[int(m.group(1))][r["Counter_Name"]][(f, r["Dispatch_Id"])] += float(r["Counter_Value"])
    per = {}
    for i, cs in acc.items():
        waves = sum(cs["SQ_WAVES"].values()) / len(cs["SQ_WAVES"])
        per[i] = {c: sum(v.values()) / len(v) / waves for c, v in cs.items() if c != "SQ_WAVES"}
    res = {}
    print(f"{'function':20s} {'VALU':>7s} {'SALU':>6s} {'f64 +*':>7s} {'fma64':>6s} {'tr64':>5s} {'tr32':>5s} "
          f"{'cvt':>5s} {'weighted':>8s}")
    for i in sorted(per):
        row = {c: v - (per[0].get(c, 0.0) if i else 0.0) for c, v in per[i].items()}
        row["issue_weighted"] = row["SQ_INSTS_VALU"] + sum(w * row.get(c, 0.0) for c, w in WEIGHT.items())
        res[NAMES[i]] = {k.replace("SQ_INSTS_", ""): round(v, 1) for k, v in row.items()}
        g = row.get
        print(f"{NAMES[i]:20s} {g('SQ_INSTS_VALU', 0):7.0f} {g('SQ_INSTS_SALU', 0):6.0f} "
              f"{g('SQ_INSTS_VALU_ADD_F64', 0) + g('SQ_INSTS_VALU_MUL_F64', 0):7.0f} {g('SQ_INSTS_VALU_FMA_F64', 0):6.0f} "
              f"{g('SQ_INSTS_VALU_TRANS_F64', 0):5.0f} {g('SQ_INSTS_VALU_TRANS_F32', 0):5.0f} "
              f"{g('SQ_INSTS_VALU_CVT', 0):5.0f} {row['issue_weighted']:8.0f}")
    if out:
        with open(out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
