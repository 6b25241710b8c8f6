"""Drop-in ``poselib.poselib.core.rotation3d`` (reference poselib/poselib/core/rotation3d.py).

Quaternions are ``[x, y, z, w]`` float32.  Every function on the retarget hot
path runs in librtg_hip.so on the MI355X; results come back on
the device of the first tensor argument (CPU in -> CPU out, like the reference).
Pure re-arrangements (conjugate, real/imag split, identity construction) are
exact and done with tensor indexing.
"""
from __future__ import annotations

import math

import numpy as np
from typing import List, Optional

import torch

from rtg import ops
from rtg.bridge import as_tensor, back, home_device

from scipy.spatial.transform import Rotation as sRot  # noqa: E402  (re-exported, as the reference does)

# the reference module has no __all__: ``from rotation3d import *`` hands its callers every public top-level name,
# imports included (parse_urdf.py uses ``List`` from it, sim scripts ``torch``).  Same set here.
__all__ = [
    "List", "Optional", "math", "torch", "sRot",
    "quat_mul", "quat_pos", "quat_abs", "quat_unit", "quat_conjugate", "quat_real", "quat_imaginary",
    "quat_norm_check", "quat_normalize", "quat_from_xyz", "quat_identity", "quat_from_angle_axis",
    "quat_from_rotation_matrix", "quat_mul_norm", "quat_rotate", "quat_inverse", "quat_identity_like",
    "quat_angle_axis", "quat_yaw_rotation", "transform_from_rotation_translation", "transform_identity",
    "transform_rotation", "transform_translation", "transform_inverse", "transform_identity_like", "transform_mul",
    "transform_apply", "rot_matrix_det", "rot_matrix_integrity_check", "rot_matrix_from_quaternion",
    "euclidean_to_rotation_matrix", "euclidean_integrity_check", "euclidean_translation", "euclidean_inverse",
    "euclidean_to_transform", "project_quat_to_axis_x", "project_quat_to_axis_y", "project_quat_to_axis_z",
    "project_quat_to_axis_xy", "project_quat_to_axis_xz", "extract_rotation_along_axis", "quat_mul_four",
    "quat_mul_three", "normalize_angle", "quat_to_angle_axis", "angle_axis_to_exp_map", "quat_to_exp_map",
    "exp_map_to_angle_axis", "exp_map_to_quat", "quat_to_eular",
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


def quat_from_xyz(xyz):
    """rotation3d.py:101-108: [xyz, 1 - |xyz|] (norm over the whole tensor: one 3-vector)."""
    dev = home_device(xyz)
    x = as_tensor(xyz)
    if x.shape[-1] != 3 or x.numel() != 3:
        raise RuntimeError("quat_from_xyz: the reference's whole-tensor norm only concatenates for one (3,) vector")
    q = ops.quat_from_xyz(x.reshape(1, 3))
    assert bool((q[:, 3] >= 0).all()), "xyz has its norm greater than 1"
    return back(q.reshape(*x.shape[:-1], 4), dev)


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


def quat_yaw_rotation(x, z_up: bool = True):
    """rotation3d.py:243-261: keep (z, w) [z_up] or (y, w), zero the rest (exact), then quat_normalize."""
    q = as_tensor(x)
    keep = [2, 3] if z_up else [1, 3]
    mask = torch.zeros(4, dtype=torch.bool, device=q.device)
    mask[keep] = True
    return quat_normalize(torch.where(mask, q, torch.zeros_like(q)))


def transform_from_rotation_translation(r: Optional[torch.Tensor] = None, t: Optional[torch.Tensor] = None):
    """rotation3d.py:264-275.  As in the reference, a missing part is built from the OTHER part's full shape
    (``quat_identity(list(t.shape))``), so only r and t together concatenate for batched inputs."""
    assert r is not None or t is not None, "rotation and translation can't be all None"
    if r is None:
        r = quat_identity(list(as_tensor(t).shape))
    if t is None:
        t = torch.zeros(list(as_tensor(r).shape) + [3])
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
    """rotation3d.py:309-314: identity transforms of x's FULL shape (the reference passes x.shape)."""
    return transform_identity(list(as_tensor(x).shape))


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


def rot_matrix_det(x):
    """rotation3d.py:338-350: a(ei - fh) - b(di - fg) + c(dh - eg)."""
    return _run(ops.rot_matrix_det, x)


def rot_matrix_integrity_check(x):
    """rotation3d.py:353-365.  The reference's orthogonality test calls ``Tensor.zeros_like()``, which does not
    exist: past the determinant assertion it always raises.  Same behaviour."""
    det = rot_matrix_det(x)
    assert bool((abs(det - 1) < 1e-3).all()), "the matrix has non-one determinant"
    raise RuntimeError("rot_matrix_integrity_check: 'Tensor' object has no attribute or method 'zeros_like' "
                       "(rotation3d.py:361, as in the reference)")


def rot_matrix_from_quaternion(quaternions):
    """rotation3d.py:398-427: [x, y, z, w] quaternions -> (..., 3, 3) with two_s = 2 / |q|^2."""
    return _run(ops.rot_matrix_from_quaternion, quaternions)


def euclidean_to_rotation_matrix(x):
    """rotation3d.py:430-435"""
    return as_tensor(x)[..., :3, :3]


def euclidean_integrity_check(x):
    """rotation3d.py:438-442"""
    x = as_tensor(x)
    euclidean_to_rotation_matrix(x)
    assert bool((x[..., 3, :3] == 0).all()), "the last row is illegal"
    assert bool((x[..., 3, 3] == 1).all()), "the last row is illegal"


def euclidean_translation(x):
    """rotation3d.py:445-450"""
    return as_tensor(x)[..., :3, 3]


def euclidean_inverse(x):
    """rotation3d.py:453-462.  The reference calls ``Tensor.zeros_like()`` (no such method) and always raises."""
    raise RuntimeError("euclidean_inverse: 'Tensor' object has no attribute or method 'zeros_like' "
                       "(rotation3d.py:458, as in the reference)")


def euclidean_to_transform(transformation_matrix):
    """rotation3d.py:465-473: [quat_from_rotation_matrix(R), t]."""
    m = as_tensor(transformation_matrix)
    return transform_from_rotation_translation(r=quat_from_rotation_matrix(euclidean_to_rotation_matrix(m)),
                                               t=euclidean_translation(m))


def project_quat_to_axis_x(batch_q):
    """rotation3d.py:479-486"""
    return _run(lambda q: ops.project_quat_to_axis(q, "x"), batch_q)


def project_quat_to_axis_y(batch_q):
    """rotation3d.py:488-495"""
    return _run(lambda q: ops.project_quat_to_axis(q, "y"), batch_q)


def project_quat_to_axis_z(batch_q):
    """rotation3d.py:497-504"""
    return _run(lambda q: ops.project_quat_to_axis(q, "z"), batch_q)


def project_quat_to_axis_xy(batch_q):
    """rotation3d.py:506-517: quat_mul(pitch about x, yaw about y)"""
    return _run(lambda q: ops.project_quat_to_axis(q, "xy"), batch_q)


def project_quat_to_axis_xz(batch_q):
    """rotation3d.py:519-530: quat_mul(pitch about x, roll about z)"""
    return _run(lambda q: ops.project_quat_to_axis(q, "xz"), batch_q)


def extract_rotation_along_axis(batch_quat, axis: int):
    """rotation3d.py:534-556: the atan2 angle of the rotation about axis 0 (x), 1 (y) or 2 (z)."""
    return _run(lambda q: ops.extract_rotation_along_axis(q, axis), batch_quat)


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


def exp_map_to_angle_axis(exp_map):
    """rotation3d.py:629-646: angle = normalize_angle(|e|), axis = e / |e|; |angle| <= 1e-5 -> (0, z)."""
    dev = home_device(exp_map)
    a, ax = ops.exp_map_to_angle_axis(as_tensor(exp_map))
    return back(a, dev), back(ax, dev)


def exp_map_to_quat(exp_map):
    """rotation3d.py:648-652: quat_from_angle_axis(*exp_map_to_angle_axis(e))."""
    return _run(ops.exp_map_to_quat, exp_map)


def quat_to_eular(q):
    """rotation3d.py:658-661: scipy ``from_quat(q).as_euler('xyz', degrees=True)`` -- evaluated in float64 on
    the device (the scipy restatement of quat_in_xyz_axis); returns a float64 numpy array like scipy."""
    t = as_tensor(q)
    out = ops.quat_as_euler(t, "xyz", degrees=True).cpu().numpy()
    if (out.reshape(-1).view(np.uint64) == np.uint64(0x7FF8000000000002)).any():   # rtg.h: scipy refuses q
        raise ValueError("Found zero norm quaternions in `quat`.")
    return out
