"""Drop-in ``retarget.spatial_transform.transform3d`` (reference retarget/spatial_transform/transform3d.py).

The reference operates on single vectors (``torch.dot`` on 1-D tensors,
:72,92,96); these accept any leading batch shape and run on the MI355X.
Results return on the device of the first tensor argument.
"""
from __future__ import annotations

import copy  # noqa: F401  (re-exported: the reference's module namespace is its star-export surface)
from typing import Dict  # noqa: F401

import numpy as np  # noqa: F401  (sim_full_body_teleop.py uses ``np`` from ``transform3d import *``)
import torch
from scipy.spatial.transform import Rotation as sRot  # noqa: F401

from poselib.poselib.core.rotation3d import *  # noqa: F401,F403  (the reference re-exports rotation3d)
from rtg import _lib, ops
from rtg.bridge import as_tensor, back, home_device
from rtg.runtime import raise_frame_error


def quat_between_two_vecs(vec1, vec2):
    """(:8-21) the rotation taking vec1 to vec2 per row: normalise([v1 x v2, 1 + v1.v2]); identity rows when the
    largest |vec1| or |vec2| in the batch is <= 1e-6 (the reference decides that over the whole batch)."""
    dev = home_device(vec1, vec2)
    return back(ops.quat_between_two_vecs(as_tensor(vec1), as_tensor(vec2)), dev)


def coord_transform(p, order: list = None, dir=None):
    """Axis permutation / sign flip (:24-29); exact, done in place on p's device."""
    p = as_tensor(p)
    if order is not None:
        p = p[..., order]
    if dir is not None:
        p = p * as_tensor(dir).to(p.device)
    return p


def _raise_if_marked(t: torch.Tensor, code: int) -> None:
    """The reference raises for the whole call when one element is refused (rtg.h rtg_frame_error); the kernels
    mark such elements with RTG_FRAME_NAN | code.  The message names the first marked element, as torch's does."""
    if not t.numel():
        return
    rows = (t.reshape(t.shape[0] if t.dim() > 1 else 1, -1).view(torch.int32) == (_lib.FRAME_NAN | code)).any(1)
    if bool(rows.any()):
        raise_frame_error(code, int(torch.nonzero(rows)[0, 0]))


def cal_joint_quat(zero_pose_local_translation, motion_local_translation):
    """Kabsch fit (:31-50): (B, n, 3) zero-pose vectors vs (B, n, 3) motion vectors -> (B, 4).  Raises torch's
    RuntimeError where a fit's matrix has a NaN entry (torch.linalg.svd, :40)."""
    dev = home_device(zero_pose_local_translation, motion_local_translation)
    q = ops.cal_joint_quat(as_tensor(zero_pose_local_translation), as_tensor(motion_local_translation))
    _raise_if_marked(q, _lib.FRAME_SVD_NONFINITE)
    return back(q, dev)


def quat_in_xyz_axis(q, seq: str = "xyz"):
    """scipy Euler split into three single-axis quaternions (:52-59).  Raises scipy's ValueError on a zero-norm or
    NaN quaternion (from_quat, :53)."""
    dev = home_device(q)
    a, b, c = ops.quat_in_xyz_axis(as_tensor(q), seq)
    _raise_if_marked(a, _lib.FRAME_ZERO_NORM_QUAT)
    return back(a, dev), back(b, dev), back(c, dev)


def proj_in_plane(v, n):
    """v - (v.n / |n|^2) n (:61-75)."""
    dev = home_device(v, n)
    return back(ops.proj_in_plane(as_tensor(v), as_tensor(n)), dev)


def radians_between_vecs(v1, v2, n):
    """Signed angle v1 -> v2 about n (:77-100)."""
    dev = home_device(v1, v2, n)
    return back(ops.radians_between_vecs(as_tensor(v1), as_tensor(v2), as_tensor(n)), dev)


def exp_map_to_quat(exp_map):
    """(:146-150) = rotation3d.exp_map_to_quat"""
    dev = home_device(exp_map)
    return back(ops.exp_map_to_quat(as_tensor(exp_map)), dev)


def quat_slerp(q0, q1, t):
    """(:152-174) spherical interpolation with the reference's shortest-arc flip and its two fallbacks
    (|sin half| < 0.001 -> midpoint, |cos half| >= 1 -> q0); t broadcasts to (..., 1)."""
    dev = home_device(q0, q1, t)
    return back(ops.quat_slerp(as_tensor(q0), as_tensor(q1), as_tensor(t)), dev)


def quat_to_dof_pos(quat, dof_axis):
    """exp-map of each quaternion, component dof_axis[k] (:176-183)."""
    q = as_tensor(quat)
    dev = q.device
    e = ops.quat_to_exp_map(q)
    idx = torch.as_tensor(list(dof_axis), device=e.device, dtype=torch.long)
    return back(e.gather(-1, idx.expand(*e.shape[:-1]).unsqueeze(-1)).squeeze(-1), dev)
