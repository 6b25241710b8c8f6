"""ctypes wrapper around ``librtg_oracle.so`` -- TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of the reference hot path (see
``rtg_oracle.c`` header for the arithmetic contract).  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may use
it, and only as the checker / CPU baseline -- never on the product path.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "librtg_oracle.so")

_f = ctypes.POINTER(ctypes.c_float)
_d = ctypes.POINTER(ctypes.c_double)
_i = ctypes.POINTER(ctypes.c_int32)
_i64 = ctypes.c_int64

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = ctypes.CDLL(LIB_PATH)
    return _lib


def _fp(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(_f)


def _c32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.float32))


def _i32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.int32))


def full_body_pos(zl, zg, body, lh, rh, precise_gripper=True, want_rot=True, kabsch_quats=None):
    """``kabsch_quats`` (B,3,4): optional injected torso/left-wrist/right-wrist Kabsch results."""
    zl, zg, body, lh, rh = map(_c32, (zl, zg, body, lh, rh))
    kq = _c32(kabsch_quats) if kabsch_quats is not None else None
    B = body.shape[0]
    dof = np.empty((B, 30), np.float32)
    lr = np.empty((B, 31, 4), np.float32) if want_rot else None
    br = np.empty((B, 59, 4), np.float32) if want_rot else None
    lib().oracle_full_body_pos_kq(_fp(zl), _fp(zg), int(precise_gripper), _fp(body), _fp(lh), _fp(rh), _i64(B),
                                  _fp(dof), _fp(lr) if want_rot else None, _fp(br) if want_rot else None,
                                  _fp(kq) if kq is not None else None)
    return dof, lr, br


def upper_body(zl, x):
    zl, x = _c32(zl), _c32(x)
    B = x.shape[0]
    dof = np.empty((B, 30), np.float32)
    lr = np.empty((B, 31, 4), np.float32)
    lib().oracle_upper_body(_fp(zl), _fp(x), _i64(B), _fp(dof), _fp(lr))
    return dof, lr


def full_body_rot(zl, brot, bpos, lh, rh):
    zl, brot, bpos, lh, rh = map(_c32, (zl, brot, bpos, lh, rh))
    B = brot.shape[0]
    dof = np.empty((B, 30), np.float32)
    lr = np.empty((B, 31, 4), np.float32)
    lib().oracle_full_body_rot(_fp(zl), _fp(brot), _fp(bpos), _fp(lh), _fp(rh), _i64(B), _fp(dof), _fp(lr))
    return dof, lr


def body_rot(parents, grot):
    p, grot = _i32(parents), _c32(grot)
    B = grot.shape[0]
    dof = np.empty((B, 30), np.float32)
    lr = np.empty((B, 31, 4), np.float32)
    lib().oracle_body_rot(p.ctypes.data_as(_i), _fp(grot), _i64(B), _fp(dof), _fp(lr))
    return dof, lr


def fk(parents, zl, local_rot, root_t):
    p, zl, lr, rt = _i32(parents), _c32(zl), _c32(local_rot), _c32(root_t)
    B, J = lr.shape[:2]
    gr = np.empty((B, J, 4), np.float32)
    gp = np.empty((B, J, 3), np.float32)
    lib().oracle_fk(p.ctypes.data_as(_i), _fp(zl), ctypes.c_int32(J), _fp(lr), _fp(rt), _i64(B), _fp(gr), _fp(gp))
    return gr, gp


def dof_fk(parents, zl, axis, dof, root_rot, root_t, lower=None, upper=None):
    """HuForwardModel.forward_kinematics: dof (B, J-1), root_rot (B, 4), root_t (B, 3); optional clip limits."""
    p, zl, ax = _i32(parents), _c32(zl), _i32(axis)
    d, rr, rt = _c32(dof), _c32(root_rot), _c32(root_t)
    B, J = d.shape[0], len(p)
    lo = _c32(lower) if lower is not None else None
    hi = _c32(upper) if upper is not None else None
    gr = np.empty((B, J, 4), np.float32)
    gp = np.empty((B, J, 3), np.float32)
    lib().oracle_dof_fk(p.ctypes.data_as(_i), _fp(zl), ctypes.c_int32(J), ax.ctypes.data_as(_i),
                        _fp(lo) if lo is not None else None, _fp(hi) if hi is not None else None,
                        _fp(d), _fp(rr), _fp(rt), _i64(B), _fp(gr), _fp(gp))
    return gr, gp


def rescale_motion(parents, zl, motion, dir=None):
    """retarget/main.py:37-47 after coord_transform(dir) (:170): motion (B, J, 3) -> (B, J, 3)."""
    p, zl, m = _i32(parents), _c32(zl), _c32(motion)
    B, J = m.shape[0], len(p)
    dv = None if dir is None else _c32(np.asarray(dir, np.float32).reshape(3))
    out = np.empty_like(m)
    lib().oracle_rescale_motion(p.ctypes.data_as(_i), _fp(zl), ctypes.c_int32(J), _fp(m), _i64(B),
                                None if dv is None else _fp(dv), _fp(out))
    return out


def quat_between(v1, v2):
    """quat_between_two_vecs (transform3d.py:8-21), batch-level identity condition included."""
    a, b = _c32(v1).reshape(-1, 3), _c32(v2).reshape(-1, 3)
    out = np.empty((a.shape[0], 4), np.float32)
    lib().oracle_quat_between(_fp(a), _fp(b), _i64(a.shape[0]), _fp(out))
    return out


def rebuild_vtrdyn(parents, zl, motion):
    """retarget/main.py:116-165 through SkeletonState's normalisation: (B, 21, 3) -> g_rot (B, 21, 4), root (B, 3)."""
    p, zl, m = _i32(parents), _c32(zl), _c32(motion)
    B, J = m.shape[0], len(p)
    gr = np.empty((B, J, 4), np.float32)
    rt = np.empty((B, 3), np.float32)
    lib().oracle_rebuild_vtrdyn(p.ctypes.data_as(_i), _fp(zl), ctypes.c_int32(J), _fp(m), _i64(B), _fp(gr), _fp(rt))
    return gr, rt


def local_rotation(parents, g_rot):
    p, g = _i32(parents), _c32(g_rot)
    B, J = g.shape[:2]
    out = np.empty_like(g)
    lib().oracle_local_rotation(p.ctypes.data_as(_i), ctypes.c_int32(J), _fp(g), _i64(B), _fp(out))
    return out


def state_fk(parents, tree_quat, local_t, local_rot, root_t):
    p, tq, lt, lr, rt = _i32(parents), _c32(tree_quat), _c32(local_t), _c32(local_rot), _c32(root_t)
    B, J = lr.shape[:2]
    gr = np.empty((B, J, 4), np.float32)
    gp = np.empty((B, J, 3), np.float32)
    lib().oracle_state_fk(p.ctypes.data_as(_i), _fp(tq), _fp(lt), ctypes.c_int32(J), _fp(lr), _fp(rt), _i64(B),
                          _fp(gr), _fp(gp))
    return gr, gp


def state_local_rotation(parents, tree_quat, g_rot):
    p, tq, g = _i32(parents), _c32(tree_quat), _c32(g_rot)
    B, J = g.shape[:2]
    out = np.empty_like(g)
    lib().oracle_state_local_rotation(p.ctypes.data_as(_i), _fp(tq), ctypes.c_int32(J), _fp(g), _i64(B), _fp(out))
    return out


def _unary(name, a, out_shape):
    a = _c32(a)
    out = np.empty(out_shape, np.float32)
    getattr(lib(), name)(_fp(a), _i64(a.shape[0]), _fp(out))
    return out


def _binary(name, a, b, out_shape):
    a, b = _c32(a), _c32(b)
    out = np.empty(out_shape, np.float32)
    getattr(lib(), name)(_fp(a), _fp(b), _i64(a.shape[0]), _fp(out))
    return out


def quat_mul(a, b):
    return _binary("oracle_quat_mul", a, b, (len(a), 4))


def quat_mul_norm(a, b):
    return _binary("oracle_quat_mul_norm", a, b, (len(a), 4))


def quat_normalize(a):
    return _unary("oracle_quat_normalize", a, (len(a), 4))


def quat_rotate(q, v):
    return _binary("oracle_quat_rotate", q, v, (len(q), 3))


def quat_from_angle_axis(angle, axis):
    return _binary("oracle_quat_from_angle_axis", angle, axis, (len(angle), 4))


def quat_from_rotation_matrix(m):
    return _unary("oracle_quat_from_rotmat", np.reshape(m, (-1, 9)), (len(m), 4))


def quat_to_exp_map(q):
    return _unary("oracle_quat_to_exp_map", q, (len(q), 3))


def quat_to_angle_axis(q):
    """rotation3d.py:587-608 -> (n,4) [angle, axis xyz]."""
    return _unary("oracle_quat_to_angle_axis", _c32(q).reshape(-1, 4), (int(np.size(q)) // 4, 4))


def normalize_angle(x):
    x = _c32(x).reshape(-1)
    out = np.empty_like(x)
    lib().oracle_normalize_angle(_fp(x), _i64(len(x)), _fp(out))
    return out


def quat_abs(q):
    q = _c32(q).reshape(-1, 4)
    out = np.empty(len(q), np.float32)
    lib().oracle_quat_abs(_fp(q), _i64(len(q)), _fp(out))
    return out


def quat_unit(q):
    return _unary("oracle_quat_unit", _c32(q).reshape(-1, 4), (int(np.size(q)) // 4, 4))


def quat_angle_axis(q):
    """rotation3d.py:230-240 -> (n,4) [angle, axis xyz]."""
    return _unary("oracle_quat_angle_axis", _c32(q).reshape(-1, 4), (int(np.size(q)) // 4, 4))


def quat_to_dof_pos(q31):
    q31 = _c32(q31)
    out = np.empty((q31.shape[0], 30), np.float32)
    lib().oracle_quat_to_dof_pos(_fp(q31), _i64(q31.shape[0]), _fp(out))
    return out


def radians_between(v1, v2, n):
    v1, v2, n = map(_c32, (v1, v2, n))
    out = np.empty(len(v1), np.float32)
    lib().oracle_radians_between(_fp(v1), _fp(v2), _fp(n), _i64(len(v1)), _fp(out))
    return out


def cal_joint_quat(Z, M):
    Z, M = _c32(Z), _c32(M)
    n, npts = Z.shape[:2]
    out = np.empty((n, 4), np.float32)
    lib().oracle_cal_joint_quat(_fp(Z), _fp(M), ctypes.c_int32(npts), _i64(n), _fp(out))
    return out


def kabsch_rotmat(A):
    """transform3d.py:40-45 as the reference computes it: MKL sgesdd restated (the oracle's Kabsch)."""
    A = _c32(np.reshape(A, (-1, 9)))
    out = np.empty_like(A)
    lib().oracle_kabsch_rotmat_sgesdd(_fp(A), _i64(len(A)), _fp(out))
    return out.reshape(-1, 3, 3)


def kabsch_rotmat_polar(A):
    """Cross-check: the exact proper-rotation polar factor in float64 (round-1 oracle), rounded to f32."""
    A = _c32(np.reshape(A, (-1, 9)))
    out = np.empty_like(A)
    lib().oracle_kabsch_rotmat(_fp(A), _i64(len(A)), _fp(out))
    return out.reshape(-1, 3, 3)


def sgesdd3(A):
    """torch.linalg.svd of (n,3,3) float32 as MKL 2024.2 sgesdd computes it -> (U, S, Vt), row-major."""
    A = _c32(np.reshape(A, (-1, 9)))
    n = len(A)
    U, S, Vt = np.empty((n, 3, 3), np.float32), np.empty((n, 3), np.float32), np.empty((n, 3, 3), np.float32)
    info = lib().oracle_sgesdd3(_fp(A), _i64(n), _fp(U), _fp(S), _fp(Vt))
    assert info == 0, "sbdsqr did not converge"
    return U, S, Vt


def kabsch_rotmat_horn(A):
    """Cross-check of the device formulation (Horn/QCP) -- not used by the oracle solvers."""
    A = _c32(np.reshape(A, (-1, 9)))
    out = np.empty_like(A)
    it = np.empty(len(A), np.int32)
    lib().oracle_kabsch_rotmat_horn(_fp(A), _i64(len(A)), _fp(out), it.ctypes.data_as(_i))
    return out.reshape(-1, 3, 3), it


def quat_in_xyz_axis(q, seq):
    q = _c32(q)
    out = np.empty((len(q), 3, 4), np.float32)
    lib().oracle_quat_in_xyz_axis(_fp(q), seq.encode(), _i64(len(q)), _fp(out))
    return out


def as_euler(q, seq):
    q = _c32(q)
    out = np.empty((len(q), 3), np.float64)
    lib().oracle_as_euler(_fp(q), seq.encode(), _i64(len(q)), out.ctypes.data_as(_d))
    return out


def shoulder_pr(v1, v0, parent):
    v1, v0, parent = map(_c32, (v1, v0, parent))
    out = np.empty((len(v1), 2, 4), np.float32)
    lib().oracle_shoulder_pr(_fp(v1), _fp(v0), _fp(parent), _i64(len(v1)), _fp(out))
    return out


def elbow_py(v1, v0, parent):
    v1, v0, parent = map(_c32, (v1, v0, parent))
    out = np.empty((len(v1), 2, 4), np.float32)
    lib().oracle_elbow_py(_fp(v1), _fp(v0), _fp(parent), _i64(len(v1)), _fp(out))
    return out


def linear_velocity(p, dt, weights=None):
    p = _c32(p)
    L, J = p.shape[-3], p.shape[-2]
    nseq = int(np.prod(p.shape[:-3])) if p.ndim > 3 else 1
    out = np.empty_like(p)
    w = None if weights is None else np.ascontiguousarray(weights, np.float64)
    R = 0 if w is None else (len(w) - 1) // 2
    lib().oracle_linear_velocity(_fp(p), _i64(nseq), _i64(L), _i64(J * 3), ctypes.c_float(dt),
                                 None if w is None else w.ctypes.data_as(_d), ctypes.c_int32(R), _fp(out))
    return out


def angular_velocity(r, dt, weights=None):
    r = _c32(r)
    L, J = r.shape[-3], r.shape[-2]
    nseq = int(np.prod(r.shape[:-3])) if r.ndim > 3 else 1
    out = np.empty(r.shape[:-1] + (3,), np.float32)
    w = None if weights is None else np.ascontiguousarray(weights, np.float64)
    R = 0 if w is None else (len(w) - 1) // 2
    lib().oracle_angular_velocity(_fp(r), _i64(nseq), _i64(L), _i64(J), ctypes.c_float(dt),
                                  None if w is None else w.ctypes.data_as(_d), ctypes.c_int32(R), _fp(out))
    return out


def atan2f(y, x):
    y, x = _c32(y), _c32(x)
    out = np.empty_like(y)
    lib().oracle_atan2f_n(_fp(y), _fp(x), _i64(len(y)), _fp(out))
    return out


# ---- the rest of the rotation3d / transform3d surface (rotation3d.py:101-108, 338-427, 479-556, 629-661;
# transform3d.py:146-174), rows of the reference's per-element arithmetic
def exp_map_to_angle_axis(e):
    """rotation3d.py:629-646 -> (n,4) [angle, axis xyz]."""
    e = _c32(e).reshape(-1, 3)
    return _unary("oracle_exp_map_to_angle_axis", e, (len(e), 4))


def exp_map_to_quat(e):
    e = _c32(e).reshape(-1, 3)
    return _unary("oracle_exp_map_to_quat", e, (len(e), 4))


def quat_slerp(q0, q1, t):
    q0, q1 = _c32(q0).reshape(-1, 4), _c32(q1).reshape(-1, 4)
    t = _c32(np.broadcast_to(np.asarray(t, np.float32).reshape(-1), (len(q0),)))
    out = np.empty((len(q0), 4), np.float32)
    lib().oracle_quat_slerp(_fp(q0), _fp(q1), _fp(t), _i64(len(q0)), _fp(out))
    return out


def quat_from_xyz(xyz):
    xyz = _c32(xyz).reshape(-1, 3)
    return _unary("oracle_quat_from_xyz", xyz, (len(xyz), 4))


def rot_matrix_det(m):
    m = _c32(m).reshape(-1, 9)
    out = np.empty(len(m), np.float32)
    lib().oracle_rot_matrix_det(_fp(m), _i64(len(m)), _fp(out))
    return out


def rot_matrix_from_quaternion(q):
    q = _c32(q).reshape(-1, 4)
    return _unary("oracle_rot_matrix_from_quat", q, (len(q), 3, 3))


def extract_rotation_along_axis(q, axis):
    q = _c32(q).reshape(-1, 4)
    out = np.empty(len(q), np.float32)
    lib().oracle_rotation_along_axis(_fp(q), ctypes.c_int32(axis), _i64(len(q)), _fp(out))
    return out


PROJECT_MODES = {"x": 0, "y": 1, "z": 2, "xy": 3, "xz": 4}


def project_quat_to_axis(q, which):
    q = _c32(q).reshape(-1, 4)
    out = np.empty((len(q), 4), np.float32)
    lib().oracle_project_quat_to_axis(_fp(q), ctypes.c_int32(PROJECT_MODES[which]), _i64(len(q)), _fp(out))
    return out


def quat_to_eular(q):
    """rotation3d.py:658-661: scipy as_euler('xyz', degrees=True) = radians * (180 / pi) (np.rad2deg)."""
    return as_euler(_c32(q).reshape(-1, 4), "xyz") * (180.0 / np.pi)


def frame_status(dof) -> np.ndarray:
    """The per-frame rtg_frame_error code (include/rtg.h) carried by a solver's dof rows: 0 for a frame the reference
    solves, else the payload of dof[:, 0] (RTG_FRAME_NAN | code) -- 1 where torch.linalg.svd raises, 2 where
    scipy's from_quat raises."""
    d0 = np.ascontiguousarray(np.asarray(dof, np.float32)[:, 0]).view(np.uint32)
    return np.where((d0 & 0xFFFFFFF0) == 0x7FC00000, d0 & 0xF, 0).astype(np.int8)
