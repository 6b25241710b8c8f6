"""Drop-in ``retarget/main.py`` motion-level prep on the MI355X.

``Retarget.rescale_motion_to_standard_size`` (main.py:37-47) and
``RetargetHuV5fromMocap._rebuild_with_vtrdyn_zero_pose`` (main.py:116-165) run
as HIP launches (``rtg_rescale_motion_f32``, ``rtg_rebuild_vtrdyn_f32``); the
rebuilt motion's velocities come from the GPU SkeletonMotion path.

``RetargetHuV5fromMocap.retarget_from_global_translation`` (main.py:169-279)
runs the same chain batched over all frames: coord_transform + rescale (one
launch), the rebuild (one launch + the SkeletonState FK of the rebuilt motion),
then the per-frame arm loop as four batched joint-map launches on the rebuilt
motion's global rotation 10 and FK'd translations (the elbow parent is
quat_mul_three, unnormalised, as in the loop), then SkeletonState(is_local=True)
-> SkeletonMotion(fps=30).  The reference ends by handing both motions to
``plot_skeleton_H`` (a matplotlib viewer); here that is a module-level hook that
does nothing unless replaced, and the two motions are also kept on the object.
"""
from __future__ import annotations

from abc import ABC

import torch

from poselib.poselib.skeleton.skeleton3d import SkeletonMotion, SkeletonState
from rtg import ops
from rtg.bridge import as_tensor, back, home_device, topology


def plot_skeleton_H(motions, *args, **kwargs):
    """Stand-in for poselib.visualization.common.plot_skeleton_H (main.py:280): the viewer is out of scope; replace
    this module attribute to receive [mocap_motion, retargeted_motion]."""
    return None


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
        """main.py:169-279 over every frame at once (GPU); returns None like the reference, which ends in
        plot_skeleton_H([mocap_motion, retargeted_motion]) (:280) -- see the module hook -- and keeps both motions
        as ``self.mocap_motion`` / ``self.retargeted_motion``."""
        dev = home_device(global_translation)
        zl = self.mocap_zero_pose.local_translation
        x = as_tensor(global_translation)
        # coord_transform(dir=[-1,-1,1]) (:170) folded into the rescale launch (:172)
        motion = self.rescale_motion_to_standard_size(x, self.mocap_zero_pose, dir=[-1.0, -1.0, 1.0])
        mocap_motion = self._rebuild_with_vtrdyn_zero_pose(motion)                       # :174
        mgr = as_tensor(mocap_motion.global_rotation)
        mgt = as_tensor(mocap_motion.global_translation)
        L = mgt.shape[0]
        gpu = mgt.device
        v0 = as_tensor(zl).to(gpu)
        r10 = mgr[:, 10].contiguous()
        arm = {}
        for side, (sh, el, wr) in (("left", (18, 19, 20)), ("right", (14, 15, 16))):
            # cal_shoulder_spherical_joint_rotation (:63-91) and cal_elbowP_and_shoulderY (:93-114)
            pitch, roll = ops.cal_shoulder_pr(mgt[:, el] - mgt[:, sh], v0[el].expand(L, 3), r10)
            parent = ops.quat_mul(ops.quat_mul(r10, pitch), roll)                           # quat_mul_three
            yaw, elbow = ops.cal_elbow_py(mgt[:, wr] - mgt[:, el], v0[wr].expand(L, 3), parent)
            arm[side] = (pitch, roll, yaw, elbow)
        J = self.target_zero_pose.num_joints
        robot_local_rotation = torch.zeros((L, J, 4), device=gpu, dtype=torch.float32)
        robot_local_rotation[..., 3] = 1.0
        for links, side in (((12, 13, 14, 15), "left"), ((21, 22, 23, 24), "right")):
            for link, q in zip(links, arm[side]):
                robot_local_rotation[:, link] = q
        robot_root_translation = torch.zeros((L, 3), device=gpu, dtype=torch.float32)
        retargeted_state = SkeletonState.from_rotation_and_root_translation(
            self.target_zero_pose.skeleton_tree, back(robot_local_rotation, dev), back(robot_root_translation, dev),
            is_local=True)
        retargeted_motion = SkeletonMotion.from_skeleton_state(retargeted_state, fps=30)
        self.mocap_motion, self.retargeted_motion = mocap_motion, retargeted_motion
        plot_skeleton_H([mocap_motion, retargeted_motion])
        return None
