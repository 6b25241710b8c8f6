"""``VtrdynFullBodyPosRetargeter`` (retarget/retarget_solver/full_body_pos_retargeter.py:17-217).

Positions-only full-body solver (the live teleop path, sim_full_body_teleop.py:115-119):
torso Kabsch fit, shoulder pitch/roll + shoulder yaw/elbow pitch plane
decompositions, wrist Kabsch fits split into XYZ Euler single-axis rotations,
finger-spread gripper -- one frame per GPU lane (``RTG_SOLVER_FULL_BODY_POS``).
"""
from __future__ import annotations

import torch

from rtg import _lib, ops
from rtg.bridge import as_tensor, back, home_device
from rtg.runtime import raise_frame_error

from retarget.retarget_solver.base_retargeter import BaseHumanoidRetargeter


class VtrdynFullBodyPosRetargeter(BaseHumanoidRetargeter):
    SOLVER_KIND = _lib.SOLVER_FULL_BODY_POS

    def __init__(self, mocap_zero_pose, target_zero_pose, precise_gripper=False, *, frame_server=None, idle_ms=100):
        super().__init__(mocap_zero_pose, target_zero_pose, precise_gripper, frame_server=frame_server,
                         idle_ms=idle_ms)
        self.precise_gripper = precise_gripper

    def retarget(self, body_global_translation, left_hand_global_translation, right_hand_global_translation):
        """One frame: body (21,3), hands (20,3) -> (local_rot (31,4), dof (30,), body_global_rotation (59,4)).
        Raises where the reference raises: RuntimeError (torch.linalg.svd of a NaN Kabsch matrix, transform3d.py:40)
        or ValueError (scipy's zero-norm quaternion, transform3d.py:53); nothing is recorded then."""
        fr, b = self._frame_runner, body_global_translation
        if fr is not None and type(b) is torch.Tensor and b.is_cpu:   # the live loop's frame: straight to the runner
            lr, dof, br = fr(b, left_hand_global_translation, right_hand_global_translation)
            if fr.status:
                raise_frame_error(fr.status)
        else:
            lr, dof, br = self._solve([body_global_translation, left_hand_global_translation,
                                       right_hand_global_translation], batched=False, want_body_rot=True)
        self._record(lr, dof)
        return lr, dof, br

    def retarget_batch(self, body_global_translation, left_hand_global_translation, right_hand_global_translation,
                       record=False, want_body_rot=False, return_ok=False):
        """B frames: (B,21,3), (B,20,3), (B,20,3) -> (local_rot (B,31,4), dof (B,30), body_rot (B,59,4) | None
        [, ok (B,)]).  Frames the reference raises on (a zero-length or axis-aligned arm segment, a straight elbow,
        a NaN point: rtg.h rtg_frame_error) come back as NaN rows with ok False; record keeps only the others."""
        lr, dof, br = self._solve([body_global_translation, left_hand_global_translation,
                                   right_hand_global_translation], batched=True, want_body_rot=want_body_rot)
        ok = self._batch_out(lr, dof, record, return_ok)
        return (lr, dof, br, ok) if return_ok else (lr, dof, br)


def cal_elbowP_and_shoulderY(v1, v0, parent_global_rotation):
    """:220-243 -> (shoulder_yaw_quat, elbow_pitch_quat)"""
    dev = home_device(v1, v0, parent_global_rotation)
    y, e = ops.cal_elbow_py(as_tensor(v1), as_tensor(v0), as_tensor(parent_global_rotation))
    return back(y, dev), back(e, dev)


def cal_shoulderPR(v1, v0, parent_global_rotation):
    """:246-278 -> (pitch_joint_quat, roll_joint_quat)"""
    dev = home_device(v1, v0, parent_global_rotation)
    p, r = ops.cal_shoulder_pr(as_tensor(v1), as_tensor(v0), as_tensor(parent_global_rotation))
    return back(p, dev), back(r, dev)
