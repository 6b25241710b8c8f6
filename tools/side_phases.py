"""Where the headline side kernel's time goes (k_solve_sides<FULL_BODY_POS>, B = 262144, SoA inputs).

Needs a build with -DRTG_EXP_TIMESTAMPS=1 (tools/build_variants.sh "ts:-DRTG_EXP_TIMESTAMPS=1", then
RTG_LIB=humanoid-real-time-retarget_amd/variants/ts.so): lane 0 of each wave of every 8th block records the 100 MHz
wall clock at the phase boundaries (rtg_solver.cuh, TS slots).  Prints, per wave side and per residency round, the
median time of each phase (us) and the spread of block start / end times.
Slots: 0 start, 1 first fit's points loaded + A formed, 2 its SVD + R done, 3 phase-1 done, 4 after the R10 hand-over
(right wave: flag seen; left wave: flag raised), 5 phase-2 done (left: wrist fit; right: both arm chains), 6 after
the left-chain hand-over, 7 Euler split + gripper done, 8 exp-map read-out done, 9 past the tile counter, 12 DOF tile
stored; 10 / 11 the left wave's second fit (A, SVD).  The tile's two waves meet at an LDS counter: the first to
arrive records 9 and 12 at once and exits (its "store" phase is 0), the second stores the tile's rows.  A slot a
wave never recorded stays 0 and is masked out of the medians.
Needs RTG_ALLOW_MEASUREMENT_BUILD=1 (RTG_EXP_TIMESTAMPS writes the clock into body_rot: a wrong-answer knob).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "humanoid-real-time-retarget_amd"))

from rtg import _lib, assets, ops  # noqa: E402
from rtg._lib import check, lib  # noqa: E402
from rtg.runtime import Solver, Topology, ptr, stream_handle  # noqa: E402

PH = [("loads_A", 0, 1), ("svd1", 1, 2), ("phase1_rest", 2, 3), ("handover1", 3, 4), ("phase2", 4, 5),
      ("handover2", 5, 6), ("after_arm", 6, 7), ("finalize", 7, 8), ("tile_counter", 8, 9), ("store", 9, 12)]


def main(B=262144, layout="soa", reps=5):
    zp = np.load(os.path.join(REPO, "tests", "golden", "zero_pose.npz"))
    S = Solver(_lib.SOLVER_FULL_BODY_POS, zp["vtrdyn_full_local_t"], zp["vtrdyn_full_global_t"],
               assets.parents("vtrdyn_full"), True)
    T = Topology(assets.parents("vtrdyn_full"), assets.local_translation("vtrdyn_full"), assets.tree_quat("vtrdyn_full"))
    body, lh, rh = ops.synth_full_body(T, B, seed=1234, layout=layout)
    dof = torch.empty((B, 30), device="cuda")
    nblk = (B + 127) // 128
    ns = (nblk + 7) // 8
    ts = torch.zeros(ns * 4 * 16 * 2, dtype=torch.int32, device="cuda")
    code = _lib.LAYOUT_SOA if layout == "soa" else _lib.LAYOUT_AOS
    runs = []
    for rep in range(reps + 2):
        ts.zero_()
        check(lib().rtg_retarget_f32(S.handle, ptr(body), ptr(lh), ptr(rh), None, B, code, ptr(dof), None, ptr(ts),
                                     stream_handle()))
        torch.cuda.synchronize()
        if rep >= 2:
            t = ts.cpu().numpy().view(np.uint32).astype(np.uint64)
            runs.append((t[0::2] | (t[1::2] << np.uint64(32))).astype(np.int64).reshape(ns, 4, 16))
    out = {"B": B, "layout": layout, "sampled_blocks": ns, "runs": len(runs)}
    per = []
    for raw in runs:
        t0 = raw[:, :, 0].min()
        R = (raw - t0) * 0.01          # us from the first wave's start
        R = np.where(raw == 0, np.nan, R)   # slots a wave never recorded
        start = R[:, :, 0].min(1)
        end = np.nanmax(R[:, :, 12], 1)
        order = np.argsort(start)
        # residency rounds: a block starts in round 2 once some earlier block has ended
        first_end = end.min()
        rnd = np.where(start < first_end, 1, 2)
        pct = lambda v: {f"p{q}": round(float(np.percentile(v, q)), 2) for q in (0, 10, 50, 90, 99, 100)}
        res = {"kernel_us": float(end.max()), "round1_blocks": int((rnd == 1).sum()),
               "start_us": {f"round{rr}": pct(start[rnd == rr]) for rr in (1, 2) if (rnd == rr).any()},
               "end_us": {f"round{rr}": pct(end[rnd == rr]) for rr in (1, 2) if (rnd == rr).any()},
               "block_us": {f"round{rr}": pct((end - start)[rnd == rr]) for rr in (1, 2) if (rnd == rr).any()},
               "round2_blocks": int((rnd == 2).sum()),
               "start_us_p50_round2": float(np.median(start[rnd == 2])) if (rnd == 2).any() else None,
               "end_us_p50_round1": float(np.median(end[rnd == 1]))}
        for rr in (1, 2):
            sel = rnd == rr
            if not sel.any():
                continue
            for side, waves in (("left", [0, 2]), ("right", [1, 3])):
                W = R[sel][:, waves].reshape(-1, 16)
                res[f"round{rr}_{side}"] = {name: float(np.nanmedian(W[:, b] - W[:, a])) for name, a, b in PH}
                if side == "left":
                    res[f"round{rr}_{side}"]["fit2_loads_A"] = float(np.nanmedian(W[:, 10] - W[:, 4]))
                    res[f"round{rr}_{side}"]["fit2_svd"] = float(np.nanmedian(W[:, 11] - W[:, 10]))
                res[f"round{rr}_{side}"]["total"] = float(np.nanmedian(W[:, 12] - W[:, 0]))
        per.append(res)
    out["per_run"] = per
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*(int(a) if a.isdigit() else a for a in sys.argv[1:]))
