"""Drop-in ``HuForwardModel`` (robot_kinematics_model/hu_forward_model.py:13-33).

Joint angles -> quat_from_angle_axis about each DOF's axis -> FK, as one HIP
launch (``rtg_dof_fk_f32``: the local rotations are built in-lane and never
stored).  The reference module imports ``motion_convert.*``, which it does not
ship; its tables are retarget/robot_config/Hu.py (33-link Hu, 32 DOFs, with
limits).  For the 31-link Hu v5 the axes are Hu_v5.Hu_DOF_AXIS; Hu_v5's limit
tables hold 32 entries for 30 DOFs, so clip_angles=True raises there (where the
reference's torch.clamp would fail to broadcast).
"""
from __future__ import annotations

import torch

from robot_kinematics_model.base_forward_model import BaseForwardModel
from rtg import ops
from rtg.bridge import home_device, topology
from rtg.runtime import DofModel


def _default_tables(num_dofs: int):
    if num_dofs == 32:
        from retarget.robot_config import Hu
        return Hu.Hu_DOF_AXIS, Hu.Hu_DOF_LOWER, Hu.Hu_DOF_UPPER
    if num_dofs == 30:
        from retarget.robot_config import Hu_v5
        return Hu_v5.Hu_DOF_AXIS, None, None
    raise ValueError(f"no Hu DOF table for {num_dofs} DOFs; pass dof_axis (and limits) explicitly")


class HuForwardModel(BaseForwardModel):
    def __init__(self, skeleton_tree, device="cuda:0", dof_axis=None, dof_lower=None, dof_upper=None):
        super().__init__(skeleton_tree, device)
        n = self.num_joints - 1
        if dof_axis is None:
            dof_axis, dof_lower, dof_upper = _default_tables(n)
        self.joint_rotation_axis = torch.eye(3)[list(dof_axis)]   # :16
        self.dof_lower = dof_lower
        self.dof_upper = dof_upper
        topo = topology(self.parent_indices, self.sk_local_translation)
        self._model = DofModel(topo, dof_axis, dof_lower, dof_upper)

    def forward_kinematics(self, motion_joint_angles, motion_root_translation, motion_root_rotation, clip_angles):
        """(L, J-1, 1) angles, (L, 3) root translation, (L, 1, 4) root rotation -> ((L, J, 4), (L, J, 3))."""
        if clip_angles and not self._model.has_limits:
            raise ValueError("clip_angles needs DOF limits with one entry per DOF")
        dev = home_device(motion_joint_angles, motion_root_translation, motion_root_rotation)
        g_rot, g_pos = ops.dof_forward_kinematics(self._model, motion_joint_angles, motion_root_rotation,
                                                  motion_root_translation, clip=bool(clip_angles))
        return g_rot.to(dev), g_pos.to(dev)

    def _clip_angles(self, motion_joint_angles):
        """:27-33, forward value: (clamp(a, lo, hi) - a) + a, elementwise on the angles' device."""
        a = motion_joint_angles
        lo = torch.as_tensor(self.dof_lower, dtype=a.dtype, device=a.device).reshape(1, -1, 1)
        hi = torch.as_tensor(self.dof_upper, dtype=a.dtype, device=a.device).reshape(1, -1, 1)
        c = torch.clamp(a.clone(), min=lo, max=hi)
        return (c - a).detach() + a
