"""Zero-pose assets shipped with the package (converted from the reference's
pickled SkeletonStates by tools/extract_assets.py without unpickling)."""
from __future__ import annotations

import os
from functools import lru_cache
from typing import Dict

import numpy as np

ASSET_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")
NAMES = ("hu_v5", "vtrdyn_full", "vtrdyn", "noitom", "hu")


@lru_cache(maxsize=None)
def load(name: str) -> Dict[str, np.ndarray]:
    if name not in NAMES:
        raise KeyError(f"unknown asset {name!r}; have {NAMES}")
    d = np.load(os.path.join(ASSET_DIR, f"{name}.npz"))
    return {k: d[k] for k in d.files}


def parents(name: str) -> np.ndarray:
    return load(name)["parent_indices"].astype(np.int64)


def local_translation(name: str) -> np.ndarray:
    return load(name)["local_translation"].astype(np.float32)


def tree_quat(name: str) -> np.ndarray:
    return load(name)["quat"].astype(np.float32)
