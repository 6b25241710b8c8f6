"""``VtrdynFullBodyRetargeter`` (retarget/retarget_solver/full_body_retargeter.py:15-177):
arm chains from positions, wrists from mocap rotations (``RTG_SOLVER_FULL_BODY_ROT``)."""
from __future__ import annotations

from rtg import _lib

from retarget.retarget_solver.base_retargeter import BaseHumanoidRetargeter
from retarget.retarget_solver.full_body_pos_retargeter import cal_elbowP_and_shoulderY, cal_shoulderPR

__all__ = ["VtrdynFullBodyRetargeter", "cal_elbowP_and_shoulderY", "cal_shoulderPR"]


class VtrdynFullBodyRetargeter(BaseHumanoidRetargeter):
    SOLVER_KIND = _lib.SOLVER_FULL_BODY_ROT

    def __init__(self, mocap_zero_pose, target_zero_pose):
        super().__init__(mocap_zero_pose, target_zero_pose)

    def retarget(self, body_global_rotation, body_global_translation, left_hand_global_rotation,
                 left_hand_global_translation, right_hand_global_rotation, right_hand_global_translation):
        """One frame -> (local_rot (31,4), dof (30,)); hand rotations are unused, as in the reference."""
        lr, dof, _ = self._solve([body_global_rotation, body_global_translation, left_hand_global_translation,
                                  right_hand_global_translation], batched=False)
        self._record(lr, dof)
        return lr, dof

    def retarget_batch(self, body_global_rotation, body_global_translation, left_hand_global_translation,
                       right_hand_global_translation, record=False, return_ok=False):
        """B frames -> (local_rot (B,31,4), dof (B,30)[, ok (B,)]); frames the reference raises on are NaN rows with
        ok False (BaseHumanoidRetargeter.frame_ok)."""
        lr, dof, _ = self._solve([body_global_rotation, body_global_translation, left_hand_global_translation,
                                  right_hand_global_translation], batched=True)
        ok = self._batch_out(lr, dof, record, return_ok)
        return (lr, dof, ok) if return_ok else (lr, dof)
