"""Deterministic synthetic mocap frames (host-side, numpy).

There is no recorded VTRDyn data in the reference snapshot (``test_motion/*.csv``
is absent), so every parity fixture and the bench use synthetic poses built the
way SURVEY.md §8(d) specifies: forward kinematics of the shipped mocap zero
pose with random local rotations, a random root, and per-point jitter.

* root yaw ~ U(-pi, pi) about +z, root translation ~ N(0, 0.1^2) m;
* spine / neck / shoulder / arm / wrist joints: axis ~ uniform S^2, angle ~ U(0, 1) rad;
* finger joints: angle ~ U(0, 1.2) rad about local y or z;
* leg joints: axis ~ S^2, angle ~ U(0, 0.5) rad (unused by the solvers);
* per-point jitter ~ N(0, (2 mm)^2); everything cast to float32 at the end.

Layouts follow the reference call sites: ``body`` (B,21,3) is
``full[[0,4,5,6,1,2,3,7,8,9,10,34,35,36,37,38,39,11,12,13,14]]``
(``full_body_pos_retargeter.py:320-321``), ``lh = full[14:34]``,
``rh = full[39:59]`` (``:322-323``).
"""
from __future__ import annotations

import os
from typing import Dict

import numpy as np

ASSET_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")

FULL_TO_BODY = [0, 4, 5, 6, 1, 2, 3, 7, 8, 9, 10, 34, 35, 36, 37, 38, 39, 11, 12, 13, 14]
LH_SLICE = slice(14, 34)
RH_SLICE = slice(39, 59)

# VTRDYN_FULL joint groups (names: retarget/robot_config/VTRDYN_FULL.py:9-69)
_FULL_SPINE_ARM = [7, 8, 9, 10, 11, 12, 13, 14, 34, 35, 36, 37, 38, 39]
_FULL_LEGS = [1, 2, 3, 4, 5, 6]
_FULL_FINGERS = list(range(15, 34)) + list(range(40, 59))
# VTRDYN (21) groups (retarget/robot_config/VTRDYN.py:2-26)
_BODY_SPINE_ARM = [7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20]
_BODY_LEGS = [1, 2, 3, 4, 5, 6]


def load_asset(name: str) -> Dict[str, np.ndarray]:
    d = np.load(os.path.join(ASSET_DIR, f"{name}.npz"))
    return {k: d[k] for k in d.files}


def _qmul(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    x1, y1, z1, w1 = np.moveaxis(a, -1, 0)
    x2, y2, z2, w2 = np.moveaxis(b, -1, 0)
    return np.stack([
        w1 * x2 + x1 * w2 + y1 * z2 - z1 * y2,
        w1 * y2 + y1 * w2 + z1 * x2 - x1 * z2,
        w1 * z2 + z1 * w2 + x1 * y2 - y1 * x2,
        w1 * w2 - x1 * x2 - y1 * y2 - z1 * z2,
    ], axis=-1)


def _qrot(q: np.ndarray, v: np.ndarray) -> np.ndarray:
    u = q[..., :3]
    w = q[..., 3:]
    t = 2.0 * np.cross(u, v)
    return v + w * t + np.cross(u, t)


def _axis_angle(axis: np.ndarray, angle: np.ndarray) -> np.ndarray:
    axis = axis / np.linalg.norm(axis, axis=-1, keepdims=True)
    h = 0.5 * angle[..., None]
    return np.concatenate([axis * np.sin(h), np.cos(h)], axis=-1)


def _random_local_rotations(rng, n, J, spine_arm, legs, fingers):
    q = np.zeros((n, J, 4))
    q[..., 3] = 1.0
    yaw = rng.uniform(-np.pi, np.pi, n)
    q[:, 0] = _axis_angle(np.tile([0.0, 0.0, 1.0], (n, 1)), yaw)
    for group, amax in ((spine_arm, 1.0), (legs, 0.5)):
        if not group:
            continue
        ax = rng.normal(size=(n, len(group), 3))
        ang = rng.uniform(0.0, amax, (n, len(group)))
        q[:, group] = _axis_angle(ax, ang)
    if fingers:
        which = rng.integers(0, 2, (n, len(fingers)))
        ax = np.zeros((n, len(fingers), 3))
        ax[which == 0, 1] = 1.0
        ax[which == 1, 2] = 1.0
        ang = rng.uniform(0.0, 1.2, (n, len(fingers)))
        q[:, fingers] = _axis_angle(ax, ang)
    return q


def _fk64(local_q, root_t, parents, local_t):
    n, J, _ = local_q.shape
    g_q = np.zeros_like(local_q)
    g_p = np.zeros((n, J, 3))
    for j in range(J):
        p = parents[j]
        if p < 0:
            g_q[:, j] = local_q[:, j]
            g_p[:, j] = root_t
        else:
            g_q[:, j] = _qmul(g_q[:, p], local_q[:, j])
            g_p[:, j] = _qrot(g_q[:, p], np.broadcast_to(local_t[j], (n, 3))) + g_p[:, p]
    g_q /= np.linalg.norm(g_q, axis=-1, keepdims=True)
    g_q *= np.where(g_q[..., 3:] < 0, -1.0, 1.0)
    return g_q, g_p


def synth_full_pose(n: int, seed: int = 1234):
    """Global positions (n,59,3) and rotations (n,59,4) of the VTRDYN_FULL skeleton."""
    rng = np.random.default_rng(seed)
    a = load_asset("vtrdyn_full")
    q = _random_local_rotations(rng, n, 59, _FULL_SPINE_ARM, _FULL_LEGS, _FULL_FINGERS)
    root = rng.normal(0.0, 0.1, (n, 3))
    g_q, g_p = _fk64(q, root, a["parent_indices"], a["local_translation"].astype(np.float64))
    g_p = g_p + rng.normal(0.0, 0.002, g_p.shape)
    return g_p.astype(np.float32), g_q.astype(np.float32)


def synth_full_body_inputs(n: int, seed: int = 1234):
    """(body (n,21,3), lh (n,20,3), rh (n,20,3)) for ``VtrdynFullBodyPosRetargeter.retarget``."""
    p, _ = synth_full_pose(n, seed)
    return (np.ascontiguousarray(p[:, FULL_TO_BODY]), np.ascontiguousarray(p[:, LH_SLICE]),
            np.ascontiguousarray(p[:, RH_SLICE]))


def synth_full_body_rot_inputs(n: int, seed: int = 1234):
    """Inputs for ``VtrdynFullBodyRetargeter.retarget``: body rot/pos (21) and hand pos (20)."""
    p, q = synth_full_pose(n, seed)
    return (np.ascontiguousarray(q[:, FULL_TO_BODY]), np.ascontiguousarray(p[:, FULL_TO_BODY]),
            np.ascontiguousarray(p[:, LH_SLICE]), np.ascontiguousarray(p[:, RH_SLICE]))


def synth_body21_pose(n: int, seed: int = 1234):
    """Global positions/rotations (n,21,...) of the VTRDYN 21-joint skeleton (zero-pose frame)."""
    rng = np.random.default_rng(seed)
    a = load_asset("vtrdyn")
    q = _random_local_rotations(rng, n, 21, _BODY_SPINE_ARM, _BODY_LEGS, [])
    root = rng.normal(0.0, 0.1, (n, 3))
    g_q, g_p = _fk64(q, root, a["parent_indices"], a["local_translation"].astype(np.float64))
    g_p = g_p + rng.normal(0.0, 0.002, g_p.shape)
    return g_p.astype(np.float32), g_q.astype(np.float32)


def synth_upper_body_inputs(n: int, seed: int = 1234) -> np.ndarray:
    """Raw VTRDyn (n,21,3) for ``HuUpperBodyFromMocapRetarget.retarget_from_global_translation``.

    The solver maps its input through ``coord_transform(dir=[-1,-1,1])``
    (``retarget_solver.py:41``); the raw frame is generated so that the mapped
    positions are the FK pose of ``vtrdyn_zero_pose``.
    """
    p, _ = synth_body21_pose(n, seed)
    return np.ascontiguousarray(p * np.array([-1.0, -1.0, 1.0], dtype=np.float32))


def random_local_quats(n: int, J: int, seed: int) -> np.ndarray:
    """Random unit quaternions with w >= 0, float32 (n,J,4) (mixed-target FK config)."""
    rng = np.random.default_rng(seed)
    q = rng.normal(size=(n, J, 4))
    q /= np.linalg.norm(q, axis=-1, keepdims=True)
    q *= np.where(q[..., 3:] < 0, -1.0, 1.0)
    return q.astype(np.float32)
