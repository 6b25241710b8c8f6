"""Batched FK / inverse FK over a parent-indexed tree, on the MI355X.

Reference: robot_kinematics_model/kinematics.py:13-63 (a Python loop over joints
with vector ops over frames).  Here one lane walks one frame's chain
(librtg_hip ``rtg_fk_f32`` / ``rtg_local_rotation_f32``); results are
bit-identical to the reference (tests/test_gpu_parity.py).
"""
from __future__ import annotations

import torch

from rtg import ops
from rtg.bridge import as_tensor, back, home_device, topology


def _zl_placeholder(J):
    return torch.zeros((J, 3))


def cal_forward_kinematics(motion_local_rotation, motion_root_translation, parent_indices,
                           zero_pose_local_translation):
    """(..., J, 4) local rotations + (..., 3) root -> ((..., J, 4) global rot, (..., J, 3) global pos)."""
    lr = as_tensor(motion_local_rotation)
    rt = as_tensor(motion_root_translation)
    dev = home_device(lr, rt)
    J = lr.shape[-2]
    lead = lr.shape[:-2]
    topo = topology(parent_indices, zero_pose_local_translation)
    rt = rt.to(torch.float32).broadcast_to(*lead, 3) if lead else rt.reshape(3)
    g_rot, g_pos = ops.forward_kinematics(topo, lr.reshape(-1, J, 4), rt.reshape(-1, 3))
    return back(g_rot.reshape(*lead, J, 4), dev), back(g_pos.reshape(*lead, J, 3), dev)


def cal_local_rotation(motion_global_rotation, parent_indices):
    """(..., J, 4) global rotations -> (..., J, 4) local rotations (root copied)."""
    g = as_tensor(motion_global_rotation)
    dev = g.device
    J = g.shape[-2]
    topo = topology(parent_indices, _zl_placeholder(J))
    loc = ops.local_rotation(topo, g.reshape(-1, J, 4))
    return back(loc.reshape(g.shape), dev)
