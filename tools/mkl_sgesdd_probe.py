"""How the oracle's / kernel's sgesdd restatement was pinned: stage-by-stage bit agreement with oneMKL.

torch.linalg.svd of a (1,3,3) float32 tensor is oneMKL 2024.2 SGESDD(JOBZ='A') (a third-party dependency of the
reference, transform3d.py:40).  libtorch_cpu.so exports MKL's internal LAPACK/BLAS entry points
(mkl_lapack_sgebrd, mkl_lapack_sbdsdc, mkl_lapack_sormbr, mkl_lapack_slarfg, mkl_lapack_slartg, ...), so each
stage of the published LAPACK algorithm can be compared in isolation with candidate float32 formulations
(association order, FMA placement).  This script prints, per stage, the fraction of random inputs on which each
candidate is bit-identical to MKL; the chosen candidate (marked *) is what oracle/rtg_oracle.c (la_gesdd3) and
csrc/rtg_math.cuh (la_gesdd3) implement.  It touches only torch's MKL on the CPU -- never the reference.

usage: python tools/mkl_sgesdd_probe.py [N]     (build container; MKL's bits depend on the host ISA)
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "oracle"))

L = ctypes.CDLL(os.path.join(os.path.dirname(torch.__file__), "lib", "libtorch_cpu.so"))
f32, f64 = np.float32, np.float64
I = lambda v: ctypes.byref(ctypes.c_int(v))           # noqa: E731
Fr = lambda v: ctypes.byref(ctypes.c_float(v))        # noqa: E731
Ch = lambda s: ctypes.c_char_p(s.encode())            # noqa: E731
P = lambda a: a.ctypes.data_as(ctypes.c_void_p)       # noqa: E731
H = ctypes.c_size_t(1)                                # Fortran hidden string length


def fma(a, b, c):
    """float32 fma via exact float64 product (double rounding only at f32 midpoints, ~2^-29 of inputs)."""
    return (np.asarray(a, f32).astype(f64) * np.asarray(b, f32).astype(f64) + np.asarray(c, f32).astype(f64)).astype(f32)


def table(name, ref, cands, chosen):
    rows = {k: float(np.mean(np.all(np.atleast_2d((v == ref).T).T.reshape(len(ref), -1), axis=1))) for k, v in cands.items()}
    print(f"{name}:")
    for k, v in rows.items():
        print(f"   {'*' if k == chosen else ' '} {k:<44s} {v:.4f}")
    return rows


def probe_scalars(N, g):
    out = {}
    # SLAPY2
    X = g.standard_normal((N, 2)).astype(f32)
    ref = np.array([ctypes.c_float(0).value for _ in range(0)] or [0.0] * N, f32)
    L.mkl_lapack_slapy2.restype = ctypes.c_float
    ref = np.array([L.mkl_lapack_slapy2(Fr(a), Fr(b)) for a, b in X], f32)
    xa, ya = np.abs(X[:, 0]), np.abs(X[:, 1])
    w, z = np.maximum(xa, ya), np.minimum(xa, ya)
    r = z / w
    out["slapy2"] = table("SLAPY2", ref, {
        "w*sqrt(1+(z/w)^2), no FMA (reference LAPACK)": w * np.sqrt(f32(1) + r * r),
        "w*sqrt(fma(r,r,1))": w * np.sqrt(fma(r, r, f32(1))),
        "sqrt(x^2+y^2) in f64": np.sqrt(X.astype(f64) ** 2 @ np.ones(2)).astype(f32)}, "w*sqrt(1+(z/w)^2), no FMA (reference LAPACK)")
    # SLARTG
    F, G = g.standard_normal(N).astype(f32), g.standard_normal(N).astype(f32)
    res = []
    for a, b in zip(F, G):
        c, s, rr = ctypes.c_float(), ctypes.c_float(), ctypes.c_float()
        L.mkl_lapack_slartg(Fr(a), Fr(b), ctypes.byref(c), ctypes.byref(s), ctypes.byref(rr))
        res.append((c.value, s.value, rr.value))
    ref = np.array(res, f32)
    cands = {}
    for nm, d in (("no FMA", np.sqrt(F * F + G * G)), ("fma(f,f,g*g)", np.sqrt(fma(F, F, G * G)))):
        c, rr = np.abs(F) / d, np.copysign(d, F)
        cands[f"LAPACK>=3.10 (c=|f|/d, s=g/r), {nm}"] = np.stack([c, G / rr, rr], 1)
        c, s, rr = F / d, G / d, d.copy()
        fl = (np.abs(F) > np.abs(G)) & (c < 0)
        c[fl], s[fl], rr[fl] = -c[fl], -s[fl], -rr[fl]
        cands[f"LAPACK<=3.9 (c=f/r, sign fix), {nm}"] = np.stack([c, s, rr], 1)
    out["slartg"] = table("SLARTG", ref, cands, "LAPACK>=3.10 (c=|f|/d, s=g/r), no FMA")
    return out


def probe_slarf(N, g):
    """SLARF('L', 3, 2) as SGEBD2 calls it (v(1) = 1): which dot order / update form."""
    v = np.ones((N, 3), f32)
    v[:, 1:] = (0.5 * g.standard_normal((N, 2))).astype(f32)
    tau = g.uniform(1, 2, N).astype(f32)
    Cm = g.standard_normal((N, 3, 2)).astype(f32)
    R = np.empty_like(Cm)
    for k in range(N):
        c = np.asfortranarray(Cm[k])
        w = np.zeros(8, f32)
        L.mkl_lapack_slarf(Ch("L"), I(3), I(2), P(v[k]), I(1), Fr(tau[k]), P(c), I(3), P(w), H)
        R[k] = c
    c0, c1, c2 = Cm[:, 0], Cm[:, 1], Cm[:, 2]
    v1, v2, t = v[:, 1:2], v[:, 2:3], tau[:, None]
    W = {"c0+(c1v1+c2v2)": c0 + (c1 * v1 + c2 * v2), "(c0+c1v1)+c2v2": (c0 + c1 * v1) + c2 * v2,
         "fma chain": fma(c2, v2, fma(c1, v1, c0))}
    U = {"fma(v,-(tau w),c)": lambda vi, w, ci: fma(vi, -(t * w), ci), "c-v*(tau w)": lambda vi, w, ci: ci - vi * (t * w),
         "fma(-(tau v),w,c)": lambda vi, w, ci: fma(-(t * vi), w, ci)}
    cands = {f"w={wn}; c={un}": np.stack([u(np.ones_like(v1), w, c0), u(v1, w, c1), u(v2, w, c2)], 1)
             for wn, w in W.items() for un, u in U.items()}
    return table("SLARF('L') in SGEBD2", R.reshape(N, -1), {k: x.reshape(N, -1) for k, x in cands.items()},
                 "w=c0+(c1v1+c2v2); c=fma(v,-(tau w),c)")


def probe_full(N, g):
    """Whole pipeline: oracle la_gesdd3 vs torch.linalg.svd, and the stage boundaries vs MKL's own stages."""
    import oracle as orc
    kinds = {
        "N(0,1) 3x3": g.standard_normal((N, 3, 3)),
        "Kabsch 5-point": np.einsum("bji,bjk->bik", g.standard_normal((N, 5, 3)), g.standard_normal((N, 5, 3))),
        "rank 2": np.einsum("bji,bjk->bik", g.standard_normal((N, 2, 3)), g.standard_normal((N, 2, 3))),
        "scale 1e-6": 1e-6 * g.standard_normal((N, 3, 3)),
    }
    out = {}
    print("SGESDD 3x3, oracle restatement vs torch.linalg.svd (U, S, Vt all bit-identical):")
    for k, A in kinds.items():
        A = A.astype(f32)
        U, S, Vt = orc.sgesdd3(A)
        same = 0
        for i in range(N):
            tu, ts, tv = (x.numpy()[0] for x in torch.linalg.svd(torch.from_numpy(A[i:i + 1])))
            same += np.array_equal(tu, U[i]) and np.array_equal(ts, S[i]) and np.array_equal(tv, Vt[i])
        out[k] = same / N
        print(f"     {k:<44s} {same / N:.4f}")
    return out


if __name__ == "__main__":
    N = int(sys.argv[1]) if len(sys.argv) > 1 else 4000
    torch.set_num_threads(1)
    g = np.random.default_rng(2026)
    res = {"cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": ")}
    res.update(probe_scalars(N, g))
    res["slarf_L"] = probe_slarf(N, g)
    res["sgesdd"] = probe_full(min(N, 2000), g)
    print(json.dumps(res))
