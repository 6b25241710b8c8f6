"""Measure the reference's own reproducibility floor across MKL code paths.

Build-container only (imports the reference through tools/refharness.py).

The reference's Kabsch fits call MKL ``sgesdd`` through ``torch.linalg.svd``
(``transform3d.py:42``).  MKL picks its kernels by CPU instruction set, and
its SVD bits differ between those code paths.  This script re-runs the
reference solvers on exactly the golden inputs (same generators and seeds as
tools/make_golden.py) with ``MKL_ENABLE_INSTRUCTIONS`` forced to AVX2 and to
SSE4_2, one subprocess each, and stores their DOFs in
``tests/golden/ref_isa_spread.npz``.  The golden fixtures themselves were
made on the default (AVX-512) path.  The spread between them is the
reference-vs-reference floor that ``tests/test_oracle_golden.py`` measures
the oracle against.

    python tools/ref_isa_spread.py            # writes the fixture
"""
from __future__ import annotations

import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden", "ref_isa_spread.npz")
ISAS = ("AVX2", "SSE4_2")
JOBS = ("full_body_pos_precise", "full_body_pos_binary", "upper_body", "full_body_rot")


def _child(path: str) -> None:
    sys.path.insert(0, HERE)
    import make_golden as mg
    import refharness as rh
    import torch
    torch.set_num_threads(1)
    ref = rh.load_reference()
    fns = {
        "full_body_pos_precise": lambda: mg.gen_full_body_pos(ref, torch, True, 512, 1234),
        "full_body_pos_binary": lambda: mg.gen_full_body_pos(ref, torch, False, 128, 4321),
        "upper_body": lambda: mg.gen_upper_body(ref, torch, 512, 2345),
        "full_body_rot": lambda: mg.gen_full_body_rot(ref, torch, 256, 3456),
    }
    np.savez(path, **{k: fns[k]()["dof"] for k in JOBS})


def main() -> None:
    if len(sys.argv) == 3 and sys.argv[1] == "--child":
        _child(sys.argv[2])
        return
    res = {}
    for isa in ISAS:
        tmp = f"/tmp/ref_isa_{isa}.npz"
        env = dict(os.environ, MKL_ENABLE_INSTRUCTIONS=isa, PYTHONDONTWRITEBYTECODE="1")
        subprocess.run([sys.executable, __file__, "--child", tmp], check=True, env=env)
        d = np.load(tmp)
        for k in JOBS:
            res[f"{k}_{isa}"] = d[k]
    np.savez_compressed(OUT, **res, isas=np.array(ISAS))
    for k in JOBS:
        gold = np.load(os.path.join(REPO, "tests", "golden", f"{k}.npz"))["dof"]
        for isa in ISAS:
            e = np.abs(res[f"{k}_{isa}"].astype(np.float64) - gold).max(axis=1)
            print(f"{k:24s} {isa:7s} max {e.max():.3g} p99 {np.quantile(e, .99):.3g} "
                  f"frames>1e-5 {(e > 1e-5).mean():.3f}")


if __name__ == "__main__":
    main()
