"""Glue between the reference-shaped Python API and the device ops.

The reference's functions take CPU float32 tensors.  The drop-in modules keep
that contract -- a CPU tensor in gives a CPU tensor out -- while all arithmetic
runs on the MI355X; device tensors stay on the device.  Topologies built from
(parent_indices, local_translation[, quat]) are uploaded once and cached.
"""
from __future__ import annotations

import hashlib
from typing import Optional, Tuple

import numpy as np
import torch

from .runtime import Topology, require_gpu


def as_tensor(x) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x
    return torch.as_tensor(np.asarray(x, dtype=np.float32))


def home_device(*xs) -> torch.device:
    """Device results are returned on: the first tensor argument's device (CPU default)."""
    for x in xs:
        if isinstance(x, torch.Tensor):
            return x.device
    return torch.device("cpu")


def back(t: torch.Tensor, dev: torch.device) -> torch.Tensor:
    return t if t.device == dev else t.to(dev)


_TOPO_CACHE: dict = {}


def _key(*arrays) -> str:
    h = hashlib.sha1()
    for a in arrays:
        if a is None:
            h.update(b"none")
            continue
        a = np.ascontiguousarray(a)
        h.update(str(a.dtype).encode() + str(a.shape).encode())
        h.update(a.tobytes())
    return h.hexdigest()


def _np(x, dtype) -> Optional[np.ndarray]:
    if x is None:
        return None
    if isinstance(x, torch.Tensor):
        x = x.detach().cpu().numpy()
    return np.ascontiguousarray(np.asarray(x, dtype=dtype))


def topology(parent_indices, local_translation, tree_quat=None) -> Topology:
    require_gpu()
    p = _np(parent_indices, np.int32)
    lt = _np(local_translation, np.float32).reshape(-1, 3)
    tq = _np(tree_quat, np.float32)
    k = _key(p, lt, tq)
    topo = _TOPO_CACHE.get(k)
    if topo is None:
        topo = Topology(p, lt, tq)
        _TOPO_CACHE[k] = topo
    return topo


def split_lead(t: torch.Tensor, tail: int) -> Tuple[torch.Size, torch.Tensor]:
    lead = t.shape[:-tail] if tail else t.shape
    return lead, t
