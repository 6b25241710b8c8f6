"""How large a domain-complete table of MKL VML's rounding would be (VERDICT r04 item 1's "if the needed table
exceeds ~1 MB, commit the attribution as the negative result").

For each VML function the solver path calls (tools/vml_attrib.py: acos at radians_between_vecs and quat_to_angle_axis,
sin / cos at quat_from_angle_axis and normalize_angle, sqrt at quat_from_rotation_matrix and quat_to_angle_axis), put
EVERY f32 of the domain the reference can feed it through torch's own vms* entry point and count, per binade, the
inputs whose VML value differs from the correctly rounded one.  A device table would need one entry per such input
(>= 4 bytes: the input's bits, the direction implied by the sign of a separate bit or list).  Build-container tool
(torch's libtorch_cpu.so, AVX-512 host); writes profiles/r05/vml_table_size.json.
"""
from __future__ import annotations

import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libtorch_cpu.so"))
MODE = ctypes.c_longlong(0x140102)
CH = 1 << 24


def bits(x):
    return int(np.float32(x).view(np.uint32))


# (vms name, numpy f64 reference, [(lo bits, hi bits)] covering the domain the reference's call sites can see)
DOMAINS = {
    "acos [-1, 1]": ("vmsAcos", np.arccos, [(0, bits(1.0) + 1), (0x80000000, bits(-1.0) + 1)]),
    "sin [-2pi, 2pi]": ("vmsSin", np.sin, [(0, bits(2 * np.pi) + 1), (0x80000000, bits(-2 * np.pi) + 1)]),
    "cos [-2pi, 2pi]": ("vmsCos", np.cos, [(0, bits(2 * np.pi) + 1), (0x80000000, bits(-2 * np.pi) + 1)]),
    "sqrt [0, 1]": ("vmsSqrt", np.sqrt, [(0, bits(1.0) + 1)]),
}


def scan(name, ref, ranges):
    f = getattr(L, name)
    f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong]
    per_exp = {}
    tot = mism = 0
    for lo, hi in ranges:
        for start in range(lo, hi, CH):
            b = np.arange(start, min(start + CH, hi), dtype=np.uint32)
            x = b.view(np.float32)
            v = np.empty_like(x)
            f(len(x), x.ctypes.data, v.ctypes.data, MODE)
            cr = ref(x.astype(np.float64)).astype(np.float32)
            bad = (v != cr) & ~(np.isnan(v) & np.isnan(cr))
            tot += len(x)
            mism += int(bad.sum())
            e = ((b[bad] >> 23) & 0xFF).astype(np.int64) - 127
            for k, c in zip(*np.unique(e, return_counts=True)):
                per_exp[int(k)] = per_exp.get(int(k), 0) + int(c)
    return tot, mism, per_exp


def main():
    out = {"about": __doc__.split("\n\n")[0], "functions": {}}
    for label, (name, ref, ranges) in DOMAINS.items():
        t0 = time.time()
        tot, mism, per_exp = scan(name, ref, ranges)
        lowest = min(per_exp) if per_exp else None
        out["functions"][label] = {"inputs": tot, "differ": mism, "differ_frac": mism / tot,
                                   "exception_list_bytes_at_4B": 4 * mism,
                                   "lowest_binade_with_a_mismatch": lowest,
                                   "differ_per_binade": dict(sorted(per_exp.items()))}
        print(label, tot, mism, f"{4 * mism / 2**20:.1f} MiB", lowest, f"{time.time() - t0:.0f}s", flush=True)
    out["total_exception_list_MiB"] = sum(v["exception_list_bytes_at_4B"] for v in out["functions"].values()) / 2**20
    os.makedirs(os.path.join(REPO, "profiles", "r05"), exist_ok=True)
    with open(os.path.join(REPO, "profiles", "r05", "vml_table_size.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print("total", out["total_exception_list_MiB"], "MiB")


if __name__ == "__main__":
    sys.exit(main())
