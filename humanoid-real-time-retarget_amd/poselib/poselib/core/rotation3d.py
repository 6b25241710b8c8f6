"""Drop-in ``poselib.poselib.core.rotation3d`` (reference poselib/poselib/core/rotation3d.py).

Quaternions are ``[x, y, z, w]`` float32.  Every function on the retarget hot
path runs in librtg_hip.so on the MI355X; results come back on
the device of the first tensor argument (CPU in -> CPU out, like the reference).
Pure re-arrangements (conjugate, real/imag split, identity construction) are
exact and done with tensor indexing.
"""
from __future__ import annotations

import math
from typing import List, Optional

import torch

from rtg import ops
from rtg.bridge import as_tensor, back, home_device

__all__ = [
    "quat_mul", "quat_pos", "quat_abs", "quat_unit", "quat_conjugate", "quat_real", "quat_imaginary",
    "quat_norm_check", "quat_normalize", "quat_identity", "quat_from_angle_axis", "quat_from_rotation_matrix",
    "quat_mul_norm", "quat_rotate", "quat_inverse", "quat_identity_like", "quat_angle_axis",
    "transform_from_rotation_translation", "transform_identity", "transform_rotation", "transform_translation",
    "transform_inverse", "transform_identity_like", "transform_mul", "transform_apply", "quat_mul_four",
    "quat_mul_three", "normalize_angle", "quat_to_angle_axis", "angle_axis_to_exp_map", "quat_to_exp_map",
]


def _run(fn, *args):
    dev = home_device(*args)
    return back(fn(*[as_tensor(a) for a in args]), dev)


def quat_mul(a, b):
    """Hamilton product, each component a left fold of four products (rotation3d.py:14-27)."""
    return _run(ops.quat_mul, a, b)


def quat_pos(x):
    """Flip quaternions with negative real part (rotation3d.py:30-38)."""
    x = as_tensor(x)
    return torch.where(x[..., 3:] < 0, -x, x)


def quat_abs(x):
    """|q|: sequential sum of squares, correctly rounded sqrt (rotation3d.py:41-47)."""
    return _run(ops.quat_abs, x)


def quat_unit(x):
    """x / max(|x|, 1e-9) (rotation3d.py:50-56)."""
    return _run(ops.quat_unit, x)


def quat_conjugate(x):
    """rotation3d.py:59-64"""
    x = as_tensor(x)
    return torch.cat([-x[..., :3], x[..., 3:]], dim=-1)


def quat_real(x):
    return as_tensor(x)[..., 3]


def quat_imaginary(x):
    return as_tensor(x)[..., :3]


def quat_norm_check(x):
    """rotation3d.py:83-89"""
    x = as_tensor(x)
    assert bool((abs(x.norm(p=2, dim=-1) - 1) < 1e-3).all()), "the quaternion is has non-1 norm"
    assert bool((x[..., 3] >= 0).all()), "the quaternion has negative real part"


def quat_normalize(q):
    """quat_unit(quat_pos(q)) (rotation3d.py:92-98)."""
    return _run(ops.quat_normalize, q)


def quat_identity(shape: List[int]):
    """Identity quaternions of ``shape`` (rotation3d.py:111-119); normalising [0,0,0,1] is exact."""
    q = torch.zeros(list(shape) + [4])
    q[..., 3] = 1.0
    return q


def quat_identity_like(x):
    return quat_identity(list(as_tensor(x).shape[:-1]))


def quat_from_angle_axis(angle, axis, degree: bool = False):
    """rotation3d.py:122-143"""
    dev = home_device(angle, axis)
    angle = as_tensor(angle)
    if degree:
        a = angle.to(torch.float32)
        angle = a / 180.0 * math.pi
    return back(ops.quat_from_angle_axis(angle, as_tensor(axis)), dev)


def quat_from_rotation_matrix(m):
    """rotation3d.py:146-193 (the four overlapping max-component branches, in order)."""
    return _run(ops.quat_from_rotation_matrix, m)


def quat_mul_norm(x, y):
    """rotation3d.py:196-202"""
    return _run(ops.quat_mul_norm, x, y)


def quat_rotate(rot, vec):
    """imag((q * [v,0]) * conj(q)) with two full Hamilton products (rotation3d.py:205-211)."""
    return _run(ops.quat_rotate, rot, vec)


def quat_inverse(x):
    """rotation3d.py:214-219"""
    return quat_conjugate(x)


def quat_angle_axis(x):
    """(angle in [0, pi], unit axis) (rotation3d.py:230-240)."""
    dev = home_device(x)
    a, ax = ops.quat_angle_axis(as_tensor(x))
    return back(a, dev), back(ax, dev)


def transform_from_rotation_translation(r: Optional[torch.Tensor] = None, t: Optional[torch.Tensor] = None):
    """rotation3d.py:264-275"""
    assert r is not None or t is not None, "rotation and translation can't be all None"
    if r is None:
        r = quat_identity(list(t.shape[:-1]))
    if t is None:
        t = torch.zeros(list(r.shape[:-1]) + [3])
    r, t = as_tensor(r), as_tensor(t)
    return torch.cat([r, t.to(r.device)], dim=-1)


def transform_identity(shape: List[int]):
    return transform_from_rotation_translation(quat_identity(shape), torch.zeros(list(shape) + [3]))


def transform_rotation(x):
    return as_tensor(x)[..., :4]


def transform_translation(x):
    return as_tensor(x)[..., 4:]


def transform_inverse(x):
    """rotation3d.py:300-306"""
    inv = quat_inverse(transform_rotation(x))
    return transform_from_rotation_translation(inv, quat_rotate(inv, -transform_translation(x)))


def transform_identity_like(x):
    return transform_identity(list(as_tensor(x).shape[:-1]))


def transform_mul(x, y):
    """rotation3d.py:317-326: (quat_mul_norm(rx, ry), quat_rotate(rx, ty) + tx)."""
    x, y = as_tensor(x), as_tensor(y)
    dev = home_device(x, y)
    r = ops.quat_mul_norm(transform_rotation(x), transform_rotation(y))
    t = ops.quat_rotate(transform_rotation(x), transform_translation(y)) + transform_translation(x).to(r.device)
    return back(torch.cat([r, t], dim=-1), dev)


def transform_apply(rot, vec):
    """rotation3d.py:329-334"""
    rot = as_tensor(rot)
    return quat_rotate(transform_rotation(rot), vec) + transform_translation(rot)


def quat_mul_four(q1, q2, q3, q4):
    """((q1*q2)*q3)*q4, no normalisation (rotation3d.py:559-567)."""
    return quat_mul(quat_mul(quat_mul(q1, q2), q3), q4)


def quat_mul_three(q1, q2, q3):
    """(q1*q2)*q3, no normalisation (rotation3d.py:570-577)."""
    return quat_mul(quat_mul(q1, q2), q3)


def normalize_angle(x):
    """atan2(sin x, cos x) (rotation3d.py:582-584)."""
    return _run(ops.normalize_angle, x)


def quat_to_angle_axis(q):
    """rotation3d.py:587-608"""
    dev = home_device(q)
    a, ax = ops.quat_to_angle_axis(as_tensor(q))
    return back(a, dev), back(ax, dev)


def angle_axis_to_exp_map(angle, axis):
    """rotation3d.py:611-617: angle[..., None] * axis (one rounding per element)."""
    angle, axis = as_tensor(angle), as_tensor(axis)
    return angle.unsqueeze(-1) * axis


def quat_to_exp_map(q):
    """rotation3d.py:620-627"""
    return _run(ops.quat_to_exp_map, q)
