"""Drop-in ``retarget/main.py`` motion-level prep on the MI355X.

``Retarget.rescale_motion_to_standard_size`` (main.py:37-47) and
``RetargetHuV5fromMocap._rebuild_with_vtrdyn_zero_pose`` (main.py:116-165) run
as HIP launches (``rtg_rescale_motion_f32``, ``rtg_rebuild_vtrdyn_f32``); the
rebuilt motion's velocities come from the GPU SkeletonMotion path.

The reference module's per-frame arm loop (``retarget_from_global_translation``,
main.py:169-279) is the prototype of ``HuUpperBodyFromMocapRetarget``
(retarget_solver.py:40-99), which ships as the batched UPPER_BODY solver; it
ends in a matplotlib viewer and is not reproduced here.
"""
from __future__ import annotations

from abc import ABC

import torch

from poselib.poselib.skeleton.skeleton3d import SkeletonMotion, SkeletonState
from rtg import ops
from rtg.bridge import back, home_device, topology


class Retarget(ABC):
    def __init__(self, mocap_zero_pose, target_zero_pose):
        self.mocap_zero_pose = mocap_zero_pose
        self.target_zero_pose = target_zero_pose

    def cal_motion_local_rotation(self):
        pass

    @staticmethod
    def rescale_motion_to_standard_size(motion_global_translation, zero_pose, dir=None):
        """(L, J, 3) -> (L, J, 3): every bone scaled to the zero pose's length, hung from the parent's rescaled
        position (main.py:37-47).  ``dir`` optionally folds in coord_transform(p, dir=...) (main.py:170)."""
        dev = home_device(motion_global_translation)
        topo = topology(zero_pose.parent_indices, zero_pose.local_translation)
        return back(ops.rescale_motion(topo, motion_global_translation, dir), dev)


class RetargetHuV5fromMocap(Retarget):
    def _rebuild_with_vtrdyn_zero_pose(self, motion_global_translation, fps=30) -> SkeletonMotion:
        """main.py:116-165: global rotations from the two Kabsch fits and quat_between_two_vecs of every bone,
        as the SkeletonState the reference builds (rotations normalised once there, done on the device), then
        SkeletonMotion.from_skeleton_state(fps) (velocities on the device)."""
        zp = self.mocap_zero_pose
        topo = topology(zp.parent_indices, zp.local_translation)
        g_rot, root = ops.rebuild_vtrdyn(topo, motion_global_translation)
        dev = home_device(motion_global_translation)
        state = SkeletonState(SkeletonState._to_state_vector(back(g_rot, dev), back(root, dev)),
                              skeleton_tree=zp.skeleton_tree, is_local=False)
        return SkeletonMotion.from_skeleton_state(state, fps=fps)

    def retarget_from_global_translation(self, global_translation):
        raise NotImplementedError(
            "main.py's per-frame prototype loop ends in a viewer; use "
            "retarget.retarget_solver.HuUpperBodyFromMocapRetarget (same joint maps, batched on the GPU)")
