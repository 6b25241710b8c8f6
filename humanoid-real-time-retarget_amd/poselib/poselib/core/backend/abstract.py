"""``Serializable`` file I/O of the poselib containers (reference poselib/poselib/core/backend/abstract.py:68-128).

Same two formats: ``.json`` (ndarrays as ``{"__ndarray__", "dtype", "shape"}``) and ``.npy`` (``np.save`` of the
``to_dict()`` mapping).  A ``.npy`` is read with the non-executing pickle walker (rtg.safe_pickle.read_npy_object)
instead of ``np.load(allow_pickle=True)``: the file's contents are data, never code.
"""
from __future__ import annotations

import json
import os

import numpy as np


class NumpyEncoder(json.JSONEncoder):
    """numpy scalars -> python numbers, ndarrays -> tagged dicts (abstract.py:32-58)."""

    def default(self, obj):
        if isinstance(obj, np.integer):
            return int(obj)
        if isinstance(obj, np.floating):
            return float(obj)
        if isinstance(obj, np.ndarray):
            return {"__ndarray__": obj.tolist(), "dtype": str(obj.dtype), "shape": obj.shape}
        return super().default(obj)


def json_numpy_obj_hook(dct):
    """Inverse of NumpyEncoder's ndarray tag (abstract.py:61-65)."""
    if isinstance(dct, dict) and "__ndarray__" in dct:
        return np.asarray(dct["__ndarray__"], dtype=dct["dtype"]).reshape(dct["shape"])
    return dct


class Serializable:
    """Subclasses implement ``to_dict()`` and the classmethod ``from_dict()``."""

    @classmethod
    def from_dict(cls, dict_repr, *args, **kwargs):
        raise NotImplementedError

    def to_dict(self):
        raise NotImplementedError

    @classmethod
    def from_file(cls, path, *args, **kwargs):
        if path.endswith(".json"):
            with open(path, "r") as f:
                d = json.load(f, object_hook=json_numpy_obj_hook)
        elif path.endswith(".npy"):
            from rtg.safe_pickle import read_npy_object
            d = read_npy_object(path)
        else:
            raise AssertionError(f"failed to load {cls.__name__} from {path}")
        assert d["__name__"] == cls.__name__, f"the file belongs to {d['__name__']}, not {cls.__name__}"
        return cls.from_dict(d, *args, **kwargs)

    def to_file(self, path: str) -> None:
        folder = os.path.dirname(path)
        if folder and not os.path.exists(folder):
            os.makedirs(folder)
        d = self.to_dict()
        d["__name__"] = type(self).__name__
        if path.endswith(".json"):
            with open(path, "w") as f:
                json.dump(d, f, cls=NumpyEncoder, indent=4)
        elif path.endswith(".npy"):
            np.save(path, d)
