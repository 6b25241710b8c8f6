"""``Mocap2HuBodyRetargeter`` (retarget/retarget_solver/body_retargeter.py:30-99):
rotation-only solver -- local rotations split by scipy Euler (``RTG_SOLVER_BODY_ROT``)."""
from __future__ import annotations

from robot_kinematics_model import cal_local_rotation
from rtg import _lib
from rtg.bridge import as_tensor
from poselib.poselib.core.rotation3d import quat_identity_like

from retarget.robot_config.Hu_v5 import Hu_DOF_AXIS
from retarget.retarget_solver.base_retargeter import BaseHumanoidRetargeter
from retarget.spatial_transform.transform3d import quat_to_dof_pos


class Mocap2HuBodyRetargeter(BaseHumanoidRetargeter):
    SOLVER_KIND = _lib.SOLVER_BODY_ROT

    def __init__(self, mocap_zero_pose, target_zero_pose):
        super().__init__(mocap_zero_pose, target_zero_pose)

    def retarget_from_pose(self, source_global_rotation):
        """One frame of global rotations (21,4) -> (local_rot (31,4), dof (30,))."""
        lr, dof, _ = self._solve([source_global_rotation], batched=False)
        self._record(lr, dof)
        return lr, dof

    def retarget_batch(self, source_global_rotation, record=False, return_ok=False):
        """B frames (B,21,4) -> (local_rot (B,31,4), dof (B,30)[, ok (B,)]); frames the reference raises on are NaN
        rows with ok False (BaseHumanoidRetargeter.frame_ok)."""
        lr, dof, _ = self._solve([source_global_rotation], batched=True)
        ok = self._batch_out(lr, dof, record, return_ok)
        return (lr, dof, ok) if return_ok else (lr, dof)

    def retarget_test(self, source_global_rotation):
        """Debug mapping of raw local rotations (:83-99)."""
        src = cal_local_rotation(as_tensor(source_global_rotation), self.source_zero_pose.parent_indices)
        lr = quat_identity_like(self.target_zero_pose.local_rotation).to(src.device)
        lr[13] = src[18]
        lr[15] = src[19]
        lr[22] = src[14]
        lr[24] = src[15]
        dof = quat_to_dof_pos(lr[1:], Hu_DOF_AXIS)
        self._record(lr, dof)
        return lr, dof
