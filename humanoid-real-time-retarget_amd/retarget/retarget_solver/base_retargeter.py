"""``BaseHumanoidRetargeter`` (retarget/retarget_solver/base_retargeter.py:15-58) on the MI355X.

Keeps the reference's per-frame accumulation API (``_motion_local_rotation`` /
``_motion_dof_pos`` lists, ``motion_*`` properties, FK cached until the length
changes) and adds batched solving: every solver runs through one
``rtg_retarget_f32`` launch whether it is handed one frame or millions.
"""
from __future__ import annotations

from abc import ABC
from typing import Optional, Sequence

import torch

from robot_kinematics_model import RobotZeroPose, cal_forward_kinematics
from rtg import _lib
from rtg.bridge import as_tensor, back, home_device
from rtg.runtime import Solver, dev_f32, frame_status, raise_frame_error


_CPU = torch.device("cpu")


class BaseHumanoidRetargeter(ABC):
    #: rtg_solver_kind of the subclass
    SOLVER_KIND: Optional[int] = None

    def __init__(self, source_zero_pose: RobotZeroPose, target_zero_pose: RobotZeroPose, precise_gripper=False, *,
                 frame_server: Optional[bool] = None, idle_ms: int = 100):
        self.source_zero_pose = source_zero_pose
        self.target_zero_pose = target_zero_pose
        self._motion_local_rotation = []
        self._motion_dof_pos = []
        self._solver = None
        self._precise = bool(precise_gripper)
        self._frame_runner = None
        self.configure_per_frame(frame_server, idle_ms)

    def configure_per_frame(self, frame_server: Optional[bool] = None, idle_ms: int = 100):
        """How single host frames are served (an addition to the reference API).

        frame_server=True (the default for FULL_BODY_POS; RTG_FRAME_SERVER=0 turns it off): a resident workgroup
        serves the frames with no launch per frame (rtg.realtime.FrameServer).  It ends after ``idle_ms`` without a
        frame, on :meth:`close`, or at interpreter exit, and relaunches itself on the next frame.  Default 100 ms,
        measured with the teleop loop's own work between frames (tools/extra_bench.py teleop_gaps,
        profiles/r05/teleop/): with 5-33 ms between frames a 5 ms server ended and relaunched every frame (60-186 us
        median per call) while a 50-200 ms one served each frame in 26-31 us (FrameGraph: 54-151 us).  While the
        server runs, a device-wide synchronize waits until it ends: close() it first.  frame_server=False, and every other
        solver kind: one launch per frame over pinned memory on a private stream (rtg.realtime.FrameGraph) --
        nothing stays resident."""
        if frame_server is None:
            import os
            frame_server = os.environ.get("RTG_FRAME_SERVER", "1") == "1"
        self.close()
        self.frame_server, self.idle_ms = bool(frame_server), int(idle_ms)

    # -- device solver (built lazily so construction works before a GPU is touched)
    @property
    def solver(self) -> Solver:
        if self._solver is None:
            if self.target_zero_pose.num_joints != 31:
                raise ValueError("the retarget solvers target the 31-link Hu v5 robot "
                                 f"(got {self.target_zero_pose.num_joints} links)")
            self._solver = Solver(self.SOLVER_KIND, self.source_zero_pose.local_translation,
                                  self.source_zero_pose.global_translation, self.source_zero_pose.parent_indices,
                                  self._precise)
        return self._solver

    def _solve(self, inputs: Sequence, batched: bool, want_body_rot=False):
        """Run the device solver on (B, ...) or single-frame inputs; returns (local_rot, dof, body_rot).
        A single frame of host inputs (the live teleop loop) goes to the resident frame server (FULL_BODY_POS) or a
        one-launch frame call over pinned memory (rtg.realtime.per_frame_runner).  A single frame the reference
        raises on raises the same exception here (rtg.h rtg_frame_error); a batch marks such frames instead."""
        x0 = inputs[0]
        host = (x0.is_cpu if type(x0) is torch.Tensor else home_device(*inputs) == _CPU) if not batched else False
        if host:
            if self._frame_runner is None:   # one runner per solver; FULL_BODY_POS always carries body_rot
                from rtg.realtime import per_frame_runner
                self._frame_runner = per_frame_runner(self.solver, self.SOLVER_KIND == _lib.SOLVER_FULL_BODY_POS,
                                                      server=self.frame_server, idle_ms=self.idle_ms)
            lr, dof, br = self._frame_runner(*inputs)
            if self._frame_runner.status:   # the frame is marked (read off the host row, no torch op)
                raise_frame_error(self._frame_runner.status)
            return lr, dof, (br if want_body_rot else None)
        dev = home_device(*inputs)
        tails = [tuple(as_tensor(x).shape[-2:]) for x in inputs]
        xs = [dev_f32(as_tensor(x).reshape(-1, *t)) for x, t in zip(inputs, tails)]
        dof, lr, br = self.solver.retarget(xs, want_local_rot=True, want_body_rot=want_body_rot)
        if not batched:
            raise_frame_error(frame_status(dof)[0].item())
            dof, lr = dof[0], lr[0]
            br = br[0] if br is not None else None
        return back(lr, dev), back(dof, dev), (back(br, dev) if br is not None else None)

    @staticmethod
    def frame_ok(dof) -> torch.Tensor:
        """Per-frame mask of a batch's dof rows (B, 30): False where the reference raises on the frame -- those rows
        are NaN and rtg.runtime.frame_status(dof) gives the exception (1: torch.linalg.svd RuntimeError,
        2: scipy ValueError, transform3d.py:40 / :53)."""
        return frame_status(as_tensor(dof)) == 0

    def _batch_out(self, lr, dof, record: bool, return_ok: bool):
        """A batch's outputs: records (like the per-frame calls) only the frames the reference returns a result
        for, and appends the ok mask when asked."""
        ok = self.frame_ok(dof) if (record or return_ok) else None
        if record:
            keep = ok.to(torch.bool)
            self._record(lr[keep], dof[keep])
        return ok

    def close(self):
        """End the per-frame runner (a resident frame server occupies its stream until it ends or idles out)."""
        g, self._frame_runner = getattr(self, "_frame_runner", None), None
        if g is not None and hasattr(g, "close"):
            g.close()

    def _record(self, local_rot, dof):
        self._motion_local_rotation.append(local_rot)
        self._motion_dof_pos.append(dof)

    # -- accumulated motion (base_retargeter.py:22-58)
    @property
    def motion_local_rotation(self):
        return torch.cat([x.reshape(-1, *x.shape[-2:]) for x in self._motion_local_rotation]).clone()

    @property
    def motion_dof_pos(self):
        return torch.cat([x.reshape(-1, x.shape[-1]) for x in self._motion_dof_pos]).clone()

    @property
    def motion_length(self):
        return sum(1 if x.dim() == 2 else x.shape[0] for x in self._motion_local_rotation)

    def _fk(self):
        lr = self.motion_local_rotation
        self._motion_global_rotation, self._motion_global_translation = cal_forward_kinematics(
            motion_local_rotation=lr, motion_root_translation=torch.zeros((self.motion_length, 3), device=lr.device),
            parent_indices=self.target_zero_pose.parent_indices,
            zero_pose_local_translation=self.target_zero_pose.local_translation)

    @property
    def motion_global_rotation(self):
        if not (hasattr(self, "_motion_global_rotation") and len(self._motion_global_rotation) == self.motion_length):
            self._fk()
        return self._motion_global_rotation.clone()

    @property
    def motion_global_translation(self):
        if not (hasattr(self, "_motion_global_translation")
                and len(self._motion_global_translation) == self.motion_length):
            self._fk()
        return self._motion_global_translation.clone()
