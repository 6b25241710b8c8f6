"""Drop-in ``poselib.poselib.skeleton.skeleton3d`` (reference poselib/poselib/skeleton/skeleton3d.py).

``SkeletonTree`` / ``SkeletonState`` / ``SkeletonMotion`` keep the reference's
attribute layout (``_node_names``, ``_parent_indices``, ``_local_translation``,
``_quat``, ``_node_indices``; ``tensor``, ``_skeleton_tree``, ``_is_local``,
``_fps``), so the reference's pickled assets unpickle into these classes
unchanged.  Forward / inverse kinematics (``global_transformation``,
``local_rotation``) and the quaternion algebra run in librtg_hip.so.

Offline tools of the reference (``from_mjcf``, ``from_fbx``, ``drop_nodes_by_names``,
``retarget_to``, ``compute_forward_vector``) are outside the hot path and not
provided.
"""
from __future__ import annotations

from collections import OrderedDict
from typing import List

import numpy as np
import torch

from rtg import ops
from rtg.bridge import as_tensor, back, topology
from rtg.safe_pickle import load_skeleton_state_arrays

from ..core.backend import Serializable
from ..core.rotation3d import quat_identity, quat_normalize

__all__ = ["SkeletonTree", "SkeletonState", "SkeletonMotion", "MotionDICT", "load_skeleton_state"]


class SkeletonTree(Serializable):
    """Parent-indexed rigid skeleton (skeleton3d.py:22-263)."""

    def __init__(self, node_names, parent_indices, local_translation, quat=None):
        ln, lp, ll = len(node_names), len(parent_indices), len(local_translation)
        assert len(set((ln, lp, ll))) == 1          # skeleton3d.py:87-88
        self._node_names = node_names
        self._parent_indices = torch.as_tensor(parent_indices).long()
        self._local_translation = as_tensor(local_translation)
        self._quat = quat_identity([len(node_names)]) if quat is None else as_tensor(quat)
        self._node_indices = {self.node_names[i]: i for i in range(len(self))}

    def __len__(self):
        return len(self.node_names)

    def __iter__(self):
        yield from self.node_names

    def __getitem__(self, item):
        return self.node_names[item]

    def __repr__(self):
        return (f"SkeletonTree(\n    node_names={self.node_names!r},\n    parent_indices={self.parent_indices!r},"
                f"\n    local_translation={self.local_translation!r}\n)")

    @property
    def node_names(self):
        return self._node_names

    @property
    def parent_indices(self):
        return self._parent_indices

    @property
    def local_translation(self):
        return self._local_translation

    @property
    def quat(self):
        return getattr(self, "_quat", None) if getattr(self, "_quat", None) is not None else quat_identity([len(self)])

    @property
    def num_joints(self):
        return len(self)

    def parent_of(self, node_name):
        return self[int(self.parent_indices[self.index(node_name)].item())]

    def index(self, node_name):
        return self._node_indices[node_name]

    def topology(self):
        """Device-resident topology of this tree (cached by content)."""
        return topology(self.parent_indices, self.local_translation, self.quat)

    @classmethod
    def from_dict(cls, dict_repr, *args, **kwargs):
        def arr(d):
            return torch.from_numpy(np.asarray(d["arr"]).astype(d["context"]["dtype"]))
        return cls(list(map(str, dict_repr["node_names"])), arr(dict_repr["parent_indices"]),
                   arr(dict_repr["local_translation"]), arr(dict_repr["quat"]) if "quat" in dict_repr else None)

    def to_dict(self):
        def d(x):
            x = x.detach().cpu().numpy()
            return {"arr": x, "context": {"dtype": x.dtype.name}}
        return OrderedDict([("node_names", self.node_names), ("parent_indices", d(self.parent_indices)),
                            ("local_translation", d(self.local_translation))])


class SkeletonState(Serializable):
    """A static pose: rotations (local or global) + root translation (skeleton3d.py:266-934)."""

    def __init__(self, tensor_backend, skeleton_tree, is_local):
        self._skeleton_tree = skeleton_tree
        self._is_local = is_local
        self.tensor = as_tensor(tensor_backend).clone()

    def __len__(self):
        return self.tensor.shape[0]

    # -- raw views of the state vector [J*4 rotations, 3 root translation]
    @property
    def rotation(self):
        J = self.num_joints
        return self.tensor[..., :J * 4].reshape(*(self.tensor.shape[:-1] + (J, 4)))

    @property
    def root_translation(self):
        J = self.num_joints
        return self.tensor[..., J * 4:J * 4 + 3]

    @property
    def is_local(self):
        return self._is_local

    @property
    def invariant_property(self):
        return {"skeleton_tree": self.skeleton_tree, "is_local": self.is_local}

    @property
    def num_joints(self):
        return self.skeleton_tree.num_joints

    @property
    def skeleton_tree(self):
        return self._skeleton_tree

    # -- kinematics
    @property
    def local_rotation(self):
        """Local rotations; for a global state, inverse FK incl. the tree-quat fix-up (skeleton3d.py:460-484)."""
        if self._is_local:
            return self.rotation
        cached = self.__dict__.get("_comp_local_rotation")
        if cached is None:
            g = self.rotation
            lead = g.shape[:-2]
            loc = ops.local_rotation(self.skeleton_tree.topology(), g.reshape(-1, self.num_joints, 4), state=True)
            cached = back(loc.reshape(*lead, self.num_joints, 4), g.device)
            self._comp_local_rotation = cached
        return cached

    @property
    def local_translation(self):
        """Tree translations with the root replaced by the root translation (skeleton3d.py:494-505)."""
        cached = self.__dict__.get("_local_translation")
        if cached is None:
            shape = tuple(self.tensor.shape[:-1]) + (self.num_joints, 3)
            cached = self.skeleton_tree.local_translation.to(self.tensor.device).broadcast_to(*shape).clone()
            cached[..., 0, :] = self.root_translation
            self._local_translation = cached
        return cached

    @property
    def local_transformation(self):
        return torch.cat([self.local_rotation, self.local_translation], dim=-1)

    @property
    def global_transformation(self):
        """FK through transform_mul with the tree pre-rotation (skeleton3d.py:402-425), on the MI355X."""
        cached = self.__dict__.get("_global_transformation")
        if cached is None:
            lr = self.local_rotation
            lead = lr.shape[:-2]
            J = self.num_joints
            rt = self.root_translation.reshape(-1, 3)
            g_rot, g_pos = ops.forward_kinematics(self.skeleton_tree.topology(), lr.reshape(-1, J, 4), rt, state=True)
            cached = back(torch.cat([g_rot, g_pos], dim=-1).reshape(*lead, J, 7), lr.device)
            self._global_transformation = cached
        return cached

    @property
    def global_rotation(self):
        if not self._is_local:
            return self.rotation
        return self.global_transformation[..., :4]

    @property
    def global_translation(self):
        return self.global_transformation[..., 4:]

    @property
    def global_root_rotation(self):
        return self.global_rotation[..., 0, :]

    @staticmethod
    def _to_state_vector(rot, rt):
        state_shape = rot.shape[:-2]
        vr = rot.reshape(*(state_shape + (-1,)))
        vt = rt.to(rot.device).broadcast_to(*state_shape + rt.shape[-1:]).reshape(*(state_shape + (-1,)))
        return torch.cat([vr, vt], dim=-1)

    @classmethod
    def from_rotation_and_root_translation(cls, skeleton_tree, r, t, is_local=True):
        """skeleton3d.py:594-617 -- rotations are normalised (on the device) first."""
        r = as_tensor(r)
        assert r.dim() > 0, "the rotation needs to have at least 1 dimension"
        r = quat_normalize(r)
        return cls(SkeletonState._to_state_vector(r, as_tensor(t)), skeleton_tree=skeleton_tree, is_local=is_local)

    @classmethod
    def zero_pose(cls, skeleton_tree):
        return cls.from_rotation_and_root_translation(skeleton_tree, skeleton_tree.quat,
                                                      torch.zeros(3, dtype=skeleton_tree.local_translation.dtype),
                                                      is_local=True)

    def local_repr(self):
        if self.is_local:
            return self
        return SkeletonState.from_rotation_and_root_translation(self.skeleton_tree, self.local_rotation,
                                                                self.root_translation, is_local=True)

    def global_repr(self):
        if not self.is_local:
            return self
        return SkeletonState.from_rotation_and_root_translation(self.skeleton_tree, self.global_rotation,
                                                                self.root_translation, is_local=False)

    def to_dict(self):
        def d(x):
            x = x.detach().cpu().numpy()
            return {"arr": x, "context": {"dtype": x.dtype.name}}
        return OrderedDict([("rotation", d(self.rotation)), ("root_translation", d(self.root_translation)),
                            ("skeleton_tree", self.skeleton_tree.to_dict()), ("is_local", self.is_local)])

    @classmethod
    def from_dict(cls, dict_repr, *args, **kwargs):
        def arr(d):
            return torch.from_numpy(np.asarray(d["arr"]).astype(d["context"]["dtype"]))
        return cls(SkeletonState._to_state_vector(arr(dict_repr["rotation"]), arr(dict_repr["root_translation"])),
                   SkeletonTree.from_dict(dict_repr["skeleton_tree"]), dict_repr["is_local"])


class SkeletonMotion(SkeletonState):
    """A state sequence with per-joint velocities appended (skeleton3d.py:935-1292)."""

    def __init__(self, tensor_backend, skeleton_tree, is_local, fps, *args, **kwargs):
        self._fps = fps
        super().__init__(tensor_backend, skeleton_tree, is_local)

    def clone(self):
        return SkeletonMotion(self.tensor.clone(), self.skeleton_tree, self._is_local, self._fps)

    @property
    def invariant_property(self):
        return {"skeleton_tree": self.skeleton_tree, "is_local": self.is_local, "fps": self.fps}

    @property
    def global_velocity(self):
        J = self.num_joints
        c = J * 4 + 3
        return self.tensor[..., c:c + J * 3].reshape(*(self.tensor.shape[:-1] + (J, 3)))

    @property
    def global_angular_velocity(self):
        J = self.num_joints
        c = J * 7 + 3
        return self.tensor[..., c:c + J * 3].reshape(*(self.tensor.shape[:-1] + (J, 3)))

    @property
    def fps(self):
        return self._fps

    @property
    def time_delta(self):
        return 1.0 / self.fps

    @property
    def global_root_velocity(self):
        return self.global_velocity[..., 0, :]

    @property
    def global_root_angular_velocity(self):
        return self.global_angular_velocity[..., 0, :]

    @classmethod
    def from_state_vector_and_velocity(cls, skeleton_tree, state_vector, global_velocity, global_angular_velocity,
                                       is_local, fps):
        state_vector = as_tensor(state_vector)
        shape = state_vector.shape[:-1]
        v = as_tensor(global_velocity).to(state_vector.device).reshape(*(shape + (-1,)))
        av = as_tensor(global_angular_velocity).to(state_vector.device).reshape(*(shape + (-1,)))
        return cls(torch.cat([state_vector, v, av], dim=-1), skeleton_tree=skeleton_tree, is_local=is_local, fps=fps)

    @classmethod
    def from_skeleton_state(cls, skeleton_state: SkeletonState, fps: int):
        """Velocities by np.gradient + gaussian_filter1d(sigma=2, nearest) over frames
        (skeleton3d.py:1026-1049, 1126-1146), computed on the MI355X."""
        assert type(skeleton_state) == SkeletonState, \
            f"expected type of {SkeletonState}, got {type(skeleton_state)}"
        dt = 1 / fps
        gv = ops.motion_velocity(skeleton_state.global_translation, dt)
        gav = ops.motion_angular_velocity(skeleton_state.global_rotation, dt)
        dev = skeleton_state.tensor.device
        return cls.from_state_vector_and_velocity(skeleton_state.skeleton_tree, skeleton_state.tensor,
                                                  back(gv, dev), back(gav, dev), skeleton_state.is_local, fps)

    @staticmethod
    def _to_state_vector(rot, rt, vel, avel):
        """[J*4 rotations, 3 root, J*3 velocities, J*3 angular velocities] (skeleton3d.py:1051-1058)."""
        shape = rot.shape[:-2]
        parts = [rot, rt.to(rot.device).broadcast_to(*shape + rt.shape[-1:]), vel.to(rot.device), avel.to(rot.device)]
        return torch.cat([x.reshape(*(shape + (-1,))) for x in parts], dim=-1)

    def to_dict(self):
        def arr(x):
            x = x.detach().cpu().numpy()
            return {"arr": x, "context": {"dtype": x.dtype.name}}
        return OrderedDict([("rotation", arr(self.rotation)), ("root_translation", arr(self.root_translation)),
                            ("global_velocity", arr(self.global_velocity)),
                            ("global_angular_velocity", arr(self.global_angular_velocity)),
                            ("skeleton_tree", self.skeleton_tree.to_dict()), ("is_local", self.is_local),
                            ("fps", self.fps)])

    @classmethod
    def from_dict(cls, dict_repr, *args, **kwargs):
        """skeleton3d.py:1061-1071"""
        def arr(d):
            return torch.from_numpy(np.asarray(d["arr"]).astype(d["context"]["dtype"]))
        return cls(SkeletonMotion._to_state_vector(arr(dict_repr["rotation"]), arr(dict_repr["root_translation"]),
                                                   arr(dict_repr["global_velocity"]),
                                                   arr(dict_repr["global_angular_velocity"])),
                   skeleton_tree=SkeletonTree.from_dict(dict_repr["skeleton_tree"]), is_local=dict_repr["is_local"],
                   fps=dict_repr["fps"])


class MotionDICT:
    """Global translations + skeleton tree, indexable by frame (skeleton3d.py:1295-1315; the viewers' input)."""

    def __init__(self, gt, sk_tree, get_state=False) -> None:
        self.global_translation = as_tensor(gt).clone()
        self.skeleton_tree = sk_tree
        if not get_state and self.global_translation.dim() == 2:
            self.global_translation = self.global_translation[None, ...]

    def clone(self):
        return MotionDICT(self.global_translation.clone(), self.skeleton_tree)

    def __getitem__(self, t):
        return MotionDICT(self.global_translation[t].clone(), self.skeleton_tree, get_state=True)

    def __len__(self):
        return self.global_translation.shape[0]


def load_skeleton_state(path: str) -> SkeletonState:
    """Load a reference ``SkeletonState`` pickle WITHOUT unpickling (opcode walker, rtg.safe_pickle)."""
    d = load_skeleton_state_arrays(path)
    tree = SkeletonTree(d["node_names"], torch.from_numpy(d["parent_indices"]),
                        torch.from_numpy(d["local_translation"]), torch.from_numpy(d["quat"]))
    return SkeletonState(torch.from_numpy(d["tensor"]), tree, d["is_local"])
