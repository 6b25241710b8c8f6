"""``HuUpperBodyFromMocapRetarget`` (retarget/retarget_solver/retarget_solver.py:27-158):
arms only, from 21-joint VTRDyn positions (``RTG_SOLVER_UPPER_BODY``)."""
from __future__ import annotations

from rtg import _lib

from retarget.retarget_solver.base_retargeter import BaseHumanoidRetargeter
from retarget.retarget_solver.full_body_pos_retargeter import cal_elbowP_and_shoulderY, cal_shoulderPR

__all__ = ["HuUpperBodyFromMocapRetarget", "cal_elbowP_and_shoulderY", "cal_shoulderPR"]


class HuUpperBodyFromMocapRetarget(BaseHumanoidRetargeter):
    SOLVER_KIND = _lib.SOLVER_UPPER_BODY

    def __init__(self, mocap_zero_pose, target_zero_pose):
        super().__init__(mocap_zero_pose, target_zero_pose)

    def _cal_shoulderPR(self, v1, v0, parent_global_rotation):
        return cal_shoulderPR(v1, v0, parent_global_rotation)

    def _cal_elbowP_and_shoulderY(self, v1, v0, parent_global_rotation):
        return cal_elbowP_and_shoulderY(v1, v0, parent_global_rotation)

    def retarget_from_global_translation(self, source_global_translation):
        """One raw VTRDyn frame (21,3) -> (local_rot (31,4), dof (30,))."""
        lr, dof, _ = self._solve([source_global_translation], batched=False)
        self._record(lr, dof)
        return lr, dof

    def retarget_batch(self, source_global_translation, record=False, return_ok=False):
        """(B,21,3) -> (local_rot (B,31,4), dof (B,30))."""
        lr, dof, _ = self._solve([source_global_translation], batched=True)
        ok = self._batch_out(lr, dof, record, return_ok)
        return (lr, dof, ok) if return_ok else (lr, dof)
