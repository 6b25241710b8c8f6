"""``BaseForwardModel`` (robot_kinematics_model/base_forward_model.py:7-14): FK bound to a tree."""
from abc import ABC

from robot_kinematics_model.kinematics import cal_forward_kinematics


class BaseForwardModel(ABC):
    def __init__(self, skeleton_tree, device="cuda:0"):
        self.sk_local_translation = skeleton_tree.local_translation
        self.parent_indices = skeleton_tree.parent_indices
        self.num_joints: int = skeleton_tree.num_joints
        self.device = device

    def forward_kinematics(self, **kwargs):
        return cal_forward_kinematics(**kwargs, parent_indices=self.parent_indices,
                                      zero_pose_local_translation=self.sk_local_translation)
