"""``RobotZeroPose`` -- topology + zero-pose translations (robot_kinematics_model/base_robot.py:24-119)."""
from __future__ import annotations

import copy
from collections import OrderedDict
from typing import Dict, Union

import torch

from poselib.poselib.skeleton.skeleton3d import SkeletonState, SkeletonTree
from robot_kinematics_model.kinematics import cal_forward_kinematics


class BaseRobot:
    def __init__(self):
        pass


class RobotZeroPose:
    def __init__(self, local_translation, global_translation, parent_indices, num_joints, node_names,
                 skeleton_tree: SkeletonTree):
        self._local_translation = local_translation
        self._global_translation = global_translation
        self._parent_indices = parent_indices
        self._num_joints = num_joints
        self._node_names = node_names
        self._global_rotation = torch.tensor([[0, 0, 0, 1.0]] * num_joints, dtype=torch.float32)
        self._local_rotation = torch.tensor([[0, 0, 0, 1.0]] * num_joints, dtype=torch.float32)
        self._skeleton_tree = skeleton_tree

    # getters clone, like the reference (:44-58)
    @property
    def local_translation(self):
        return self._local_translation.clone()

    @property
    def global_translation(self):
        return self._global_translation.clone()

    @property
    def global_rotation(self):
        return self._global_rotation.clone()

    @property
    def local_rotation(self):
        return self._local_rotation.clone()

    @property
    def parent_indices(self):
        return self._parent_indices.clone()

    @property
    def num_joints(self):
        return self._num_joints

    @property
    def num_dofs(self):
        return self.num_joints - 1

    @property
    def node_names(self):
        return self._node_names

    @property
    def skeleton_tree(self):
        return copy.deepcopy(self._skeleton_tree)

    @classmethod
    def from_urdf(cls, urdf_path):
        """base_robot.py:71-81: the zero pose of a URDF through the reference's own parser,
        ``retarget.utils.parse_urdf.parse_urdf`` (urdfpy ``link_fk`` -> SkeletonTree.from_dict -> SkeletonState
        .zero_pose, both drop-in classes here).  That module is not replaced: it comes from the reference checkout
        the drop-in overlays, imported on first use so that a deployment without urdfpy can still
        import this module.  Raises ImportError only when the parser (or urdfpy) cannot be imported."""
        try:
            from retarget.utils.parse_urdf import parse_urdf
        except ImportError as e:
            raise ImportError("RobotZeroPose.from_urdf needs the reference's retarget.utils.parse_urdf (and urdfpy): "
                              "overlay the drop-in onto a reference checkout, or build the zero pose with "
                              f"from_skeleton_state / from_asset ({e})") from e
        robot_zero_pose, _link_mesh_file_names = parse_urdf(urdf_path)
        return cls(local_translation=robot_zero_pose.local_translation,
                   global_translation=robot_zero_pose.global_translation,
                   parent_indices=robot_zero_pose.skeleton_tree.parent_indices,
                   num_joints=robot_zero_pose.skeleton_tree.num_joints,
                   node_names=robot_zero_pose.skeleton_tree.node_names,
                   skeleton_tree=robot_zero_pose.skeleton_tree)

    @classmethod
    def from_skeleton_state(cls, skeleton_state: SkeletonState):
        return cls(local_translation=skeleton_state.local_translation,
                   global_translation=skeleton_state.global_translation,
                   parent_indices=skeleton_state.skeleton_tree.parent_indices,
                   num_joints=skeleton_state.skeleton_tree.num_joints,
                   node_names=skeleton_state.skeleton_tree.node_names,
                   skeleton_tree=skeleton_state.skeleton_tree)

    @classmethod
    def from_asset(cls, name: str):
        """Zero pose from the package's converted assets ('hu_v5', 'vtrdyn_full', 'vtrdyn', 'noitom', 'hu')."""
        from rtg import assets
        a = assets.load(name)
        tree = SkeletonTree([str(s) for s in a["node_names"]], torch.from_numpy(a["parent_indices"]),
                            torch.from_numpy(a["local_translation"].astype("float32")),
                            torch.from_numpy(a["quat"].astype("float32")))
        return cls.from_skeleton_state(SkeletonState(torch.from_numpy(a["tensor"].astype("float32")), tree,
                                                     bool(a["is_local"])))

    @classmethod
    def from_dict(cls, robot_dict: Union[Dict, OrderedDict], is_local=False):
        if is_local:
            robot_dict["global_translation"] = cls.cal_global_translation(robot_dict["local_translation"],
                                                                          robot_dict["parent_indices"])
        else:
            robot_dict["local_translation"] = cls.cal_local_translation(robot_dict["global_translation"],
                                                                        robot_dict["parent_indices"])
        return cls(**robot_dict)

    @staticmethod
    def cal_local_translation(global_translation, parent_indices):
        local_translation = global_translation.clone()
        local_translation[1:] -= global_translation[parent_indices[1:]]
        return local_translation

    @staticmethod
    def cal_global_translation(local_translation, parent_indices):
        raise NotImplementedError   # as in the reference (:104-106)

    def rebuild_pose_by_local_rotation(self, local_rotation):
        """FK of the zero pose under new local rotations (:107-116)."""
        global_rotation, self._global_translation = cal_forward_kinematics(
            motion_local_rotation=local_rotation, motion_root_translation=self.global_translation[0],
            parent_indices=self.parent_indices, zero_pose_local_translation=self.local_translation)
        self._local_translation = self.cal_local_translation(self.global_translation, self.parent_indices)
        self._skeleton_tree._local_translation = self.local_translation
        return global_rotation

    def get_sk_zero_pose(self):
        return SkeletonState.zero_pose(self.skeleton_tree)
