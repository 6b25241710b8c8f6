"""Drop-in ``retarget.spatial_transform.transform3d`` (reference retarget/spatial_transform/transform3d.py).

The reference operates on single vectors (``torch.dot`` on 1-D tensors,
:72,92,96); these accept any leading batch shape and run on the MI355X.
Results return on the device of the first tensor argument.
"""
from __future__ import annotations

import torch

from poselib.poselib.core.rotation3d import *  # noqa: F401,F403  (the reference re-exports rotation3d)
from rtg import ops
from rtg.bridge import as_tensor, back, home_device


def coord_transform(p, order: list = None, dir=None):
    """Axis permutation / sign flip (:24-29); exact, done in place on p's device."""
    p = as_tensor(p)
    if order is not None:
        p = p[..., order]
    if dir is not None:
        p = p * as_tensor(dir).to(p.device)
    return p


def cal_joint_quat(zero_pose_local_translation, motion_local_translation):
    """Kabsch fit (:31-50): (B, n, 3) zero-pose vectors vs (B, n, 3) motion vectors -> (B, 4)."""
    dev = home_device(zero_pose_local_translation, motion_local_translation)
    return back(ops.cal_joint_quat(as_tensor(zero_pose_local_translation), as_tensor(motion_local_translation)), dev)


def quat_in_xyz_axis(q, seq: str = "xyz"):
    """scipy Euler split into three single-axis quaternions (:52-59)."""
    dev = home_device(q)
    a, b, c = ops.quat_in_xyz_axis(as_tensor(q), seq)
    return back(a, dev), back(b, dev), back(c, dev)


def proj_in_plane(v, n):
    """v - (v.n / |n|^2) n (:61-75)."""
    dev = home_device(v, n)
    return back(ops.proj_in_plane(as_tensor(v), as_tensor(n)), dev)


def radians_between_vecs(v1, v2, n):
    """Signed angle v1 -> v2 about n (:77-100)."""
    dev = home_device(v1, v2, n)
    return back(ops.radians_between_vecs(as_tensor(v1), as_tensor(v2), as_tensor(n)), dev)


def quat_to_dof_pos(quat, dof_axis):
    """exp-map of each quaternion, component dof_axis[k] (:176-183)."""
    q = as_tensor(quat)
    dev = q.device
    e = ops.quat_to_exp_map(q)
    idx = torch.as_tensor(list(dof_axis), device=e.device, dtype=torch.long)
    return back(e.gather(-1, idx.expand(*e.shape[:-1]).unsqueeze(-1)).squeeze(-1), dev)
