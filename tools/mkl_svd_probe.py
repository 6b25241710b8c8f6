"""Does torch.linalg.svd (MKL sgesdd) give the same bits on this host as in
the build container?

The reference's Kabsch fit (``transform3d.py:40-48``) is torch.linalg.svd on a
(1,3,3) float32 matrix.  ``--write`` stores U,S,Vt for 1024 seeded matrices,
one call each like the reference, in tests/golden/mkl_svd_probe.npz (build
container, AVX-512 Xeon).  Without ``--write`` it recomputes them on the current
host and prints the fraction of bit-identical matrices and the max |diff|.  It
touches only torch on the CPU, never the reference.
"""
import json
import os
import platform
import sys

import numpy as np
import torch

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                   "mkl_svd_probe.npz")


def run(n=1024):
    g = np.random.default_rng(7)
    A = g.standard_normal((n, 3, 3)).astype(np.float32)
    res = []
    for i in range(n):
        U, S, Vt = torch.linalg.svd(torch.from_numpy(A[i:i + 1]))
        res.append(np.concatenate([U.numpy().ravel(), S.numpy().ravel(), Vt.numpy().ravel()]))
    return A, np.stack(res)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


if __name__ == "__main__":
    torch.set_num_threads(1)
    A, r = run()
    if "--write" in sys.argv:
        np.savez_compressed(OUT, A=A, usv=r, cpu=np.array(cpu_model()))
    else:
        if "--save" in sys.argv:
            np.save(sys.argv[sys.argv.index("--save") + 1], r)
        ref = np.load(OUT)
        assert np.array_equal(ref["A"], A)
        same = np.all(ref["usv"] == r, axis=1)
        print(json.dumps({"cpu_here": cpu_model(), "cpu_fixture": str(ref["cpu"]),
                          "mkl_env": os.environ.get("MKL_ENABLE_INSTRUCTIONS", "default"),
                          "svd_bit_identical_frac": float(same.mean()),
                          "max_abs_diff": float(np.abs(ref["usv"] - r).max())}))
