"""``TensorUtils`` / ``tensor_to_dict`` (reference poselib/poselib/core/tensor_utils.py:15-45): the
``{"arr", "context": {"dtype"}}`` mapping of a tensor used by the skeleton containers' to_dict / from_dict."""
from collections import OrderedDict  # noqa: F401  (re-exported like the reference)

import torch

from .backend import Serializable

__all__ = ["OrderedDict", "Serializable", "TensorUtils", "tensor_to_dict", "torch"]


class TensorUtils(Serializable):
    @classmethod
    def from_dict(cls, dict_repr, *args, **kwargs):
        return torch.from_numpy(dict_repr["arr"].astype(dict_repr["context"]["dtype"]))

    def to_dict(self):
        return NotImplemented


def tensor_to_dict(x):
    x_np = x.numpy()
    return {"arr": x_np, "context": {"dtype": x_np.dtype.name}}
