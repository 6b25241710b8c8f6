"""Functional device ops over the C ABI (batched forms of the reference's functions).

Each function takes tensors (host or device; moved to the current HIP device as
contiguous float32) and returns device tensors.  Reference semantics are cited
per op; all arithmetic happens in librtg_hip.so.
"""
from __future__ import annotations

import ctypes
import functools
from typing import Sequence

import torch

from . import _lib
from ._lib import check, lib
from .runtime import Topology, dev_f32, layout_code, ptr, require_gpu, stream_handle


def _flat(t: torch.Tensor, tail: int) -> torch.Tensor:
    return t.reshape(-1, tail) if tail else t.reshape(-1)


def _quat_op(op, a, b=None, c=None, a_tail=4, b_tail=4, c_tail=3, out_tail=4):
    a = dev_f32(a)
    lead = a.shape[:-1] if a_tail else a.shape
    n = int(torch.Size(lead).numel())
    af = _flat(a, a_tail)
    bf = None if b is None else _flat(dev_f32(b).expand(*lead, *( (b_tail,) if b_tail else ())).contiguous(), b_tail)
    cf = None if c is None else _flat(dev_f32(c).expand(*lead, *((c_tail,) if c_tail else ())).contiguous(), c_tail)
    out_shape = tuple(lead) + ((out_tail,) if isinstance(out_tail, int) and out_tail else tuple(out_tail or ()))
    out = torch.empty(out_shape, device=a.device, dtype=torch.float32)
    check(lib().rtg_quat_op_f32(op, ptr(af), ptr(bf), ptr(cf), n, ptr(out), stream_handle()))
    return out


def _bcast(a, b, ta, tb):
    a, b = dev_f32(a), dev_f32(b)
    lead = torch.broadcast_shapes(a.shape[:-1], b.shape[:-1])
    return a.expand(*lead, ta).contiguous(), b.expand(*lead, tb).contiguous()


def quat_mul(a, b):
    """rotation3d.py:14-27"""
    a, b = _bcast(a, b, 4, 4)
    return _quat_op(_lib.OP_QUAT_MUL, a, b)


def quat_mul_norm(a, b):
    """rotation3d.py:196-202"""
    a, b = _bcast(a, b, 4, 4)
    return _quat_op(_lib.OP_QUAT_MUL_NORM, a, b)


def quat_normalize(q):
    """rotation3d.py:92-98"""
    return _quat_op(_lib.OP_QUAT_NORMALIZE, q)


def quat_inverse(q):
    """rotation3d.py:214-219"""
    return _quat_op(_lib.OP_QUAT_INVERSE, q)


def quat_rotate(q, v):
    """rotation3d.py:205-211"""
    q, v = _bcast(q, v, 4, 3)
    return _quat_op(_lib.OP_QUAT_ROTATE, q, v, b_tail=3, out_tail=3)


def quat_from_angle_axis(angle, axis):
    """rotation3d.py:122-143 (angle (...), axis (...,3))"""
    angle = dev_f32(angle)
    axis = dev_f32(axis)
    lead = torch.broadcast_shapes(angle.shape, axis.shape[:-1])
    angle = angle.expand(lead).contiguous()
    axis = axis.expand(*lead, 3).contiguous()
    n = int(torch.Size(lead).numel())
    out = torch.empty(tuple(lead) + (4,), device=angle.device, dtype=torch.float32)
    check(lib().rtg_quat_op_f32(_lib.OP_QUAT_FROM_ANGLE_AXIS, ptr(angle), ptr(axis), None, n, ptr(out),
                                stream_handle()))
    return out


def quat_from_rotation_matrix(m):
    """rotation3d.py:146-193 (m (...,3,3))"""
    m = dev_f32(m, (3, 3), "m")
    lead = m.shape[:-2]
    n = int(torch.Size(lead).numel())
    out = torch.empty(tuple(lead) + (4,), device=m.device, dtype=torch.float32)
    check(lib().rtg_quat_op_f32(_lib.OP_QUAT_FROM_ROTMAT, ptr(m), None, None, n, ptr(out), stream_handle()))
    return out


def quat_to_exp_map(q):
    """rotation3d.py:620-627"""
    return _quat_op(_lib.OP_QUAT_TO_EXP_MAP, q, out_tail=3)


def quat_to_angle_axis(q):
    """rotation3d.py:587-608 -> (angle (...), axis (...,3))"""
    r = _quat_op(_lib.OP_QUAT_TO_ANGLE_AXIS, q, out_tail=4)
    return r[..., 0], r[..., 1:]


def quat_abs(q):
    """rotation3d.py:41-47"""
    return _quat_op(_lib.OP_QUAT_ABS, q, out_tail=0)


def quat_unit(q):
    """rotation3d.py:50-56"""
    return _quat_op(_lib.OP_QUAT_UNIT, q)


def quat_angle_axis(q):
    """rotation3d.py:230-240 -> (angle in [0, pi] (...), unit axis (...,3))"""
    r = _quat_op(_lib.OP_QUAT_ANGLE_AXIS, q, out_tail=4)
    return r[..., 0], r[..., 1:]


def normalize_angle(x):
    """rotation3d.py:582-584 (atan2 with glibc atan2f semantics: the reference's <32-element path)"""
    x = dev_f32(x)
    out = torch.empty_like(x)
    check(lib().rtg_quat_op_f32(_lib.OP_NORMALIZE_ANGLE, ptr(x), None, None, x.numel(), ptr(out), stream_handle()))
    return out


def radians_between_vecs(v1, v2, n):
    """transform3d.py:77-100, batched over leading dims"""
    v1, v2, n = dev_f32(v1), dev_f32(v2), dev_f32(n)
    lead = torch.broadcast_shapes(v1.shape[:-1], v2.shape[:-1], n.shape[:-1])
    v1, v2, n = (t.expand(*lead, 3).contiguous() for t in (v1, v2, n))
    cnt = int(torch.Size(lead).numel())
    out = torch.empty(tuple(lead), device=v1.device, dtype=torch.float32)
    check(lib().rtg_quat_op_f32(_lib.OP_RADIANS_BETWEEN, ptr(v1), ptr(v2), ptr(n), cnt, ptr(out), stream_handle()))
    return out


def proj_in_plane(v, n):
    """transform3d.py:61-75, batched"""
    nn = dev_f32(n)
    if bool((torch.linalg.norm(nn, dim=-1) <= 1e-6).any()):
        raise AssertionError("proj_in_plane: plane normal has (near) zero length")   # transform3d.py:70
    v, nn = _bcast(v, nn, 3, 3)
    return _quat_op(_lib.OP_PROJ_IN_PLANE, v, nn, a_tail=3, b_tail=3, out_tail=3)


def quat_to_dof_pos_hu(local_rot):
    """transform3d.py:176-183 with Hu_DOF_AXIS over local_rot[..., 1:, :] (local_rot (...,31,4))"""
    lr = dev_f32(local_rot, (31, 4), "local_rot")
    lead = lr.shape[:-2]
    n = int(torch.Size(lead).numel())
    out = torch.empty(tuple(lead) + (30,), device=lr.device, dtype=torch.float32)
    check(lib().rtg_quat_op_f32(_lib.OP_QUAT_TO_DOF_POS, ptr(lr), None, None, n, ptr(out), stream_handle()))
    return out


def cal_shoulder_pr(v1, v0, parent):
    """full_body_pos_retargeter.py:246-278, batched: returns (pitch (...,4), roll (...,4))"""
    v1, v0, parent = dev_f32(v1), dev_f32(v0), dev_f32(parent)
    lead = torch.broadcast_shapes(v1.shape[:-1], v0.shape[:-1], parent.shape[:-1])
    v1, v0, parent = v1.expand(*lead, 3).contiguous(), v0.expand(*lead, 3).contiguous(), parent.expand(*lead, 4).contiguous()
    n = int(torch.Size(lead).numel())
    out = torch.empty(tuple(lead) + (2, 4), device=v1.device, dtype=torch.float32)
    check(lib().rtg_quat_op_f32(_lib.OP_SHOULDER_PR, ptr(v1), ptr(v0), ptr(parent), n, ptr(out), stream_handle()))
    return out[..., 0, :], out[..., 1, :]


def cal_elbow_py(v1, v0, parent):
    """full_body_pos_retargeter.py:220-243, batched: returns (shoulder_yaw, elbow_pitch)"""
    v1, v0, parent = dev_f32(v1), dev_f32(v0), dev_f32(parent)
    lead = torch.broadcast_shapes(v1.shape[:-1], v0.shape[:-1], parent.shape[:-1])
    v1, v0, parent = v1.expand(*lead, 3).contiguous(), v0.expand(*lead, 3).contiguous(), parent.expand(*lead, 4).contiguous()
    n = int(torch.Size(lead).numel())
    out = torch.empty(tuple(lead) + (2, 4), device=v1.device, dtype=torch.float32)
    check(lib().rtg_quat_op_f32(_lib.OP_ELBOW_PY, ptr(v1), ptr(v0), ptr(parent), n, ptr(out), stream_handle()))
    return out[..., 0, :], out[..., 1, :]


def cal_joint_quat(zero_vectors, motion_vectors):
    """transform3d.py:31-50 (Kabsch).  (..., n, 3) x (..., n, 3) -> (..., 4)"""
    Z, M = dev_f32(zero_vectors), dev_f32(motion_vectors)
    lead = torch.broadcast_shapes(Z.shape[:-2], M.shape[:-2])
    npts = int(Z.shape[-2])
    if M.shape[-2] != npts:
        raise ValueError("cal_joint_quat: point counts differ")
    Z = Z.expand(*lead, npts, 3).contiguous()
    M = M.expand(*lead, npts, 3).contiguous()
    n = int(torch.Size(lead).numel())
    out = torch.empty(tuple(lead) + (4,), device=Z.device, dtype=torch.float32)
    check(lib().rtg_cal_joint_quat_f32(ptr(Z), ptr(M), npts, n, ptr(out), stream_handle()))
    return out


def quat_in_xyz_axis(q, seq: str = "xyz"):
    """transform3d.py:52-59: three single-axis quaternions (each (...,4))."""
    q = dev_f32(q, (4,), "q")
    lead = q.shape[:-1]
    n = int(torch.Size(lead).numel())
    out = torch.empty(tuple(lead) + (3, 4), device=q.device, dtype=torch.float32)
    check(lib().rtg_quat_in_xyz_axis_f32(ptr(q), seq.encode(), n, ptr(out), stream_handle()))
    return out[..., 0, :], out[..., 1, :], out[..., 2, :]


def forward_kinematics(topo: Topology, local_rot, root_t, state: bool = False):
    """kinematics.py:13-39 (state=False) / SkeletonState FK skeleton3d.py:402-425 (state=True)."""
    J = topo.num_joints
    lr = dev_f32(local_rot, (J, 4), "local_rot")
    lead = lr.shape[:-2]
    rt = dev_f32(root_t, (3,), "root_t").expand(*lead, 3).contiguous()
    B = int(torch.Size(lead).numel())
    g_rot = torch.empty(tuple(lead) + (J, 4), device=lr.device, dtype=torch.float32)
    g_pos = torch.empty(tuple(lead) + (J, 3), device=lr.device, dtype=torch.float32)
    fn = lib().rtg_state_fk_f32 if state else lib().rtg_fk_f32
    check(fn(topo.handle, ptr(lr), ptr(rt), B, ptr(g_rot), ptr(g_pos), stream_handle()))
    return g_rot, g_pos


def local_rotation(topo: Topology, g_rot, state: bool = False):
    """kinematics.py:41-63 (state=False) / SkeletonState.local_rotation skeleton3d.py:460-484."""
    J = topo.num_joints
    g = dev_f32(g_rot, (J, 4), "g_rot")
    B = int(torch.Size(g.shape[:-2]).numel())
    out = torch.empty_like(g)
    fn = lib().rtg_state_local_rotation_f32 if state else lib().rtg_local_rotation_f32
    check(fn(topo.handle, ptr(g), B, ptr(out), stream_handle()))
    return out


def dof_forward_kinematics(model, dof, root_rot, root_t, clip: bool = False):
    """HuForwardModel.forward_kinematics (hu_forward_model.py:17-33): joint angles (..., J-1) [or (..., J-1, 1)],
    root rotation (..., 4) [or (..., 1, 4)], root translation (..., 3) -> g_rot (..., J, 4), g_pos (..., J, 3)."""
    def _t(x):
        return x if isinstance(x, torch.Tensor) else torch.as_tensor(x)

    n = model.num_dofs
    d = _t(dof)
    if d.dim() >= 2 and d.shape[-1] == 1 and d.shape[-2] == n:
        d = d[..., 0]
    d = dev_f32(d, (n,), "motion_joint_angles")
    lead = d.shape[:-1]
    rr = _t(root_rot)
    if rr.dim() >= 2 and rr.shape[-2] == 1 and rr.shape[-1] == 4:
        rr = rr[..., 0, :]
    rr = dev_f32(rr, (4,), "motion_root_rotation").expand(*lead, 4).contiguous()
    rt = dev_f32(root_t, (3,), "motion_root_translation").expand(*lead, 3).contiguous()
    B = int(torch.Size(lead).numel())
    J = n + 1
    g_rot = torch.empty(tuple(lead) + (J, 4), device=d.device, dtype=torch.float32)
    g_pos = torch.empty(tuple(lead) + (J, 3), device=d.device, dtype=torch.float32)
    check(lib().rtg_dof_fk_f32(model.handle, ptr(d), ptr(rr), ptr(rt), B, int(bool(clip)), ptr(g_rot), ptr(g_pos),
                               stream_handle()))
    return g_rot, g_pos


def rescale_motion(topo: Topology, motion, dir=None):
    """Retarget.rescale_motion_to_standard_size (retarget/main.py:37-47) after coord_transform(dir) (:170)."""
    J = topo.num_joints
    m = dev_f32(motion, (J, 3), "motion_global_translation")
    B = int(torch.Size(m.shape[:-2]).numel())
    out = torch.empty_like(m)
    d = None
    if dir is not None:
        import numpy as np
        dv = np.ascontiguousarray(np.asarray(dir.cpu() if isinstance(dir, torch.Tensor) else dir, np.float32).reshape(3))
        d = dv.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
    check(lib().rtg_rescale_motion_f32(topo.handle, ptr(m), B, d, ptr(out), stream_handle()))
    return out


def quat_between_two_vecs(v1, v2):
    """transform3d.py:8-21 (batch-level identity branch included): (..., 3) x (..., 3) -> (..., 4)."""
    a = dev_f32(v1, (3,), "vec1")
    b = dev_f32(v2, (3,), "vec2")
    if a.shape != b.shape:
        a, b = torch.broadcast_tensors(a, b)
        a, b = a.contiguous(), b.contiguous()
    n = int(torch.Size(a.shape[:-1]).numel())
    out = torch.empty(tuple(a.shape[:-1]) + (4,), device=a.device, dtype=torch.float32)
    ws = torch.empty(2, device=a.device, dtype=torch.float32)
    check(lib().rtg_quat_between_f32(ptr(a), ptr(b), n, ptr(out), ptr(ws), stream_handle()))
    return out


def rebuild_vtrdyn(topo: Topology, motion):
    """RetargetHuV5fromMocap._rebuild_with_vtrdyn_zero_pose (retarget/main.py:116-165) up to its SkeletonState:
    (B, 21, 3) rescaled positions -> (global rotations (B, 21, 4), root translation (B, 3))."""
    J = topo.num_joints
    m = dev_f32(motion, (J, 3), "motion_global_translation")
    B = int(m.shape[0])
    g_rot = torch.empty((B, J, 4), device=m.device, dtype=torch.float32)
    root = torch.empty((B, 3), device=m.device, dtype=torch.float32)
    ws = torch.empty(J, device=m.device, dtype=torch.float32)
    check(lib().rtg_rebuild_vtrdyn_f32(topo.handle, ptr(m), B, ptr(g_rot), ptr(root), ptr(ws), stream_handle()))
    return g_rot, root


def forward_kinematics_multi(segments: Sequence[tuple]):
    """One launch over several (topology, local_rot (B,J,4), root_t (B,3)) segments.

    Returns a list of (g_rot, g_pos) per segment.
    """
    require_gpu()
    if len(segments) > _lib.MAX_SEGMENTS:
        raise ValueError(f"at most {_lib.MAX_SEGMENTS} segments per launch")
    segs, keep, outs = _fk_segments(segments)
    check(lib().rtg_fk_multi_f32(segs, len(segments), stream_handle()))
    return outs


def _fk_segments(segments):
    """ctypes FK segment table with per-segment shape checks: local_rot (B, J, 4) and a root translation that
    broadcasts to (B, 3) -- a 2-D local_rot would otherwise make the kernel read B*J*4 floats of a J*4 buffer."""
    segs = (_lib.FkSegment * max(1, len(segments)))()
    keep, outs = [], []
    for i, (topo, lr, rt) in enumerate(segments):
        J = topo.num_joints
        lr = dev_f32(lr, (J, 4), "local_rot")
        if lr.dim() != 3:
            raise ValueError(f"segment {i}: local_rot must be (B, {J}, 4), got {tuple(lr.shape)}")
        B = int(lr.shape[0])
        rt = dev_f32(rt, (3,), "root_t")
        if rt.dim() > 2 or (rt.dim() == 2 and rt.shape[0] not in (1, B)):
            raise ValueError(f"segment {i}: root_t must broadcast to ({B}, 3), got {tuple(rt.shape)}")
        rt = rt.expand(B, 3).contiguous()   # a (3,) / (1,3) root translation is shared by every frame
        g_rot = torch.empty((B, J, 4), device=lr.device, dtype=torch.float32)
        g_pos = torch.empty((B, J, 3), device=lr.device, dtype=torch.float32)
        segs[i] = _lib.FkSegment(topo.handle.value, lr.data_ptr(), rt.data_ptr(), g_rot.data_ptr(), g_pos.data_ptr(), B)
        keep += [lr, rt]
        outs.append((g_rot, g_pos))
    return segs, keep, outs


def _inv_segments(segments):
    segs = (_lib.LocalRotationSegment * max(1, len(segments)))()
    keep, outs = [], []
    for i, (topo, g) in enumerate(segments):
        J = topo.num_joints
        g = dev_f32(g, (J, 4), "g_rot")
        if g.dim() != 3:
            raise ValueError(f"segment {i}: g_rot must be (B, {J}, 4), got {tuple(g.shape)}")
        out = torch.empty_like(g)
        segs[i] = _lib.LocalRotationSegment(topo.handle.value, g.data_ptr(), out.data_ptr(), int(g.shape[0]))
        keep.append(g)
        outs.append(out)
    return segs, keep, outs


def local_rotation_multi(segments: Sequence[tuple]):
    """One launch of cal_local_rotation (kinematics.py:41-63) over several (topology, g_rot (B,J,4)) segments."""
    require_gpu()
    if len(segments) > _lib.MAX_SEGMENTS:
        raise ValueError(f"at most {_lib.MAX_SEGMENTS} segments per launch")
    segs, keep, outs = _inv_segments(segments)
    check(lib().rtg_local_rotation_multi_f32(segs, len(segments), stream_handle()))
    return outs


def kinematics_multi(fk_segments: Sequence[tuple], inv_segments: Sequence[tuple]):
    """FK segments (topology, local_rot, root_t) and inverse-FK segments (topology, g_rot) in ONE launch
    (BASELINE config 5).  Returns ([(g_rot, g_pos)...], [local_rot...])."""
    require_gpu()
    if len(fk_segments) + len(inv_segments) > _lib.MAX_SEGMENTS:
        raise ValueError(f"at most {_lib.MAX_SEGMENTS} segments per launch")
    fsegs, keep, fouts = _fk_segments(fk_segments)
    isegs, ikeep, iouts = _inv_segments(inv_segments)
    check(lib().rtg_kinematics_multi_f32(fsegs, len(fk_segments), isegs, len(inv_segments), stream_handle()))
    return fouts, iouts


@functools.lru_cache(maxsize=8)
def gaussian_taps(sigma: float = 2.0, truncate: float = 4.0):
    """scipy.ndimage.gaussian_filter1d's taps (float64), as the reference applies them (sigma 2).  Cached (the
    velocity calls take them every time); the array is read-only."""
    import numpy as np
    radius = int(truncate * float(sigma) + 0.5)
    try:
        from scipy.ndimage._filters import _gaussian_kernel1d
        w = _gaussian_kernel1d(sigma, 0, radius)[::-1]
    except Exception:  # noqa: BLE001 -- same formula without scipy
        x = np.arange(-radius, radius + 1)
        w = np.exp(-0.5 / (sigma * sigma) * x ** 2)
        w = (w / w.sum())[::-1]
    w = np.ascontiguousarray(w, dtype=np.float64)
    w.flags.writeable = False
    return w, radius


def _time_axis_view(x, tail):
    x = dev_f32(x)
    if x.dim() < 1 + tail:
        raise ValueError("need a frame axis")
    L = int(x.shape[-1 - tail])
    nseq = int(torch.Size(x.shape[:-1 - tail]).numel())
    return x, nseq, L


def motion_velocity(p, dt: float, smooth: bool = True, sigma: float = 2.0):
    """SkeletonMotion._compute_velocity (skeleton3d.py:1126-1135): p (..., L, J, 3) -> (..., L, J, 3).  ``sigma``:
    the smoothing filter's (the reference's is 2; radius 4 sigma, at most 16)."""
    x, nseq, L = _time_axis_view(p, 2)
    S = int(x.shape[-2] * x.shape[-1])
    out = torch.empty_like(x)
    tmp = torch.empty_like(x) if smooth else None
    w, r = gaussian_taps(sigma) if smooth else (None, 0)
    check(lib().rtg_linear_velocity_f32(ptr(x), nseq, L, S, ctypes.c_float(dt),
                                        w.ctypes.data_as(ctypes.c_void_p) if smooth else None, r, ptr(tmp), ptr(out),
                                        stream_handle()))
    return out


def motion_angular_velocity(r, dt: float, smooth: bool = True, sigma: float = 2.0):
    """SkeletonMotion._compute_angular_velocity (skeleton3d.py:1137-1146): r (..., L, J, 4) -> (..., L, J, 3).
    ``sigma`` as in motion_velocity."""
    x, nseq, L = _time_axis_view(r, 2)
    J = int(x.shape[-2])
    out = torch.empty(tuple(x.shape[:-1]) + (3,), device=x.device, dtype=torch.float32)
    tmp = torch.empty_like(out) if smooth else None
    w, rad = gaussian_taps(sigma) if smooth else (None, 0)
    check(lib().rtg_angular_velocity_f32(ptr(x), nseq, L, J, ctypes.c_float(dt),
                                         w.ctypes.data_as(ctypes.c_void_p) if smooth else None, rad, ptr(tmp),
                                         ptr(out), stream_handle()))
    return out


def synth_full_body(topo_full: Topology, B: int, seed: int = 1234, frame_offset: int = 0, want_rot: bool = False,
                    out=None, layout="aos"):
    """Synthetic VTRDyn frames generated on the device (rtg_synth_full_body_f32), as (B,P,C) rows (``"aos"``)
    or (P,C,B) component planes (``"soa"``)."""
    dev = require_gpu()
    code = layout_code(layout)
    shp = (lambda P, C: (P, C, B)) if code == _lib.LAYOUT_SOA else (lambda P, C: (B, P, C))
    if out is None:
        body = torch.empty(shp(21, 3), device=dev, dtype=torch.float32)
        lh = torch.empty(shp(20, 3), device=dev, dtype=torch.float32)
        rh = torch.empty(shp(20, 3), device=dev, dtype=torch.float32)
    else:
        body, lh, rh = out
        for t, want in ((body, shp(21, 3)), (lh, shp(20, 3)), (rh, shp(20, 3))):
            if tuple(t.shape) != want or not t.is_contiguous() or t.dtype != torch.float32:
                raise ValueError(f"synth_full_body: output buffer {tuple(t.shape)} != {want}")
    rot = torch.empty(shp(21, 4), device=dev, dtype=torch.float32) if want_rot else None
    check(lib().rtg_synth_full_body_f32(topo_full.handle, ctypes.c_uint64(seed), frame_offset, B, code, ptr(body),
                                        ptr(lh), ptr(rh), ptr(rot), stream_handle()))
    return (body, lh, rh, rot) if want_rot else (body, lh, rh)


# ---- the rest of the rotation3d / transform3d surface (rtg_quat_op_f32 ops 18-31, rtg_quat_as_euler_f64)
def exp_map_to_angle_axis(e):
    """rotation3d.py:629-646 -> (angle (...), axis (...,3))"""
    r = _quat_op(_lib.OP_EXP_MAP_TO_ANGLE_AXIS, e, a_tail=3, out_tail=4)
    return r[..., 0], r[..., 1:]


def exp_map_to_quat(e):
    """rotation3d.py:648-652 / transform3d.py:146-150"""
    return _quat_op(_lib.OP_EXP_MAP_TO_QUAT, e, a_tail=3, out_tail=4)


def quat_slerp(q0, q1, t):
    """transform3d.py:152-174: q0, q1 (...,4), t broadcastable to (...,1) -> (...,4)"""
    q0, q1 = _bcast(q0, q1, 4, 4)
    t = dev_f32(t)
    if t.dim() >= 1 and t.shape[-1] == 1 and t.dim() == q0.dim():
        t = t[..., 0]
    t = t.expand(q0.shape[:-1]).contiguous()
    return _quat_op(_lib.OP_QUAT_SLERP, q0, q1, t, c_tail=0)


def quat_from_xyz(xyz):
    """rotation3d.py:101-108 per row: (...,3) -> (...,4) [xyz, 1 - |xyz|]"""
    return _quat_op(_lib.OP_QUAT_FROM_XYZ, xyz, a_tail=3, out_tail=4)


def rot_matrix_det(m):
    """rotation3d.py:338-350: (...,3,3) -> (...)"""
    m = dev_f32(m, (3, 3), "m")
    lead = m.shape[:-2]
    out = torch.empty(tuple(lead), device=m.device, dtype=torch.float32)
    check(lib().rtg_quat_op_f32(_lib.OP_ROT_MATRIX_DET, ptr(m), None, None, int(torch.Size(lead).numel()), ptr(out),
                                stream_handle()))
    return out


def rot_matrix_from_quaternion(q):
    """rotation3d.py:398-427: (...,4) -> (...,3,3)"""
    return _quat_op(_lib.OP_ROT_MATRIX_FROM_QUAT, q, out_tail=(3, 3))


def extract_rotation_along_axis(q, axis: int):
    """rotation3d.py:534-556: (n,4) -> (n)"""
    if axis not in (0, 1, 2):
        raise ValueError("Invalid axis. Axis must be 0 (x), 1 (y), or 2 (z).")
    return _quat_op(_lib.OP_ROTATION_ALONG_X + axis, q, out_tail=0)


def project_quat_to_axis(q, which: str):
    """project_quat_to_axis_{x,y,z,xy,xz} (rotation3d.py:479-530): (n,4) -> (n,4)"""
    return _quat_op(_lib.OP_PROJECT_QUAT[which], q)


def quat_as_euler(q, seq: str, degrees: bool = False):
    """scipy Rotation.from_quat(q).as_euler(seq, degrees) in float64 on the device: (...,4) -> (...,3) f64."""
    q = dev_f32(q, (4,), "q")
    lead = q.shape[:-1]
    out = torch.empty(tuple(lead) + (3,), device=q.device, dtype=torch.float64)
    check(lib().rtg_quat_as_euler_f64(ptr(q), seq.encode(), int(bool(degrees)), int(torch.Size(lead).numel()),
                                      ptr(out), stream_handle()))
    return out


def box_probe() -> dict:
    """rtg_box_probe (rtg.h): the current GPU's shader clock under load, f32 FMA rate and HBM copy bandwidth,
    measured now -- recorded beside every bench line so throughput from different boxes can be compared."""
    require_gpu()
    out = (ctypes.c_double * _lib.PROBE_FIELDS)()
    check(lib().rtg_box_probe(out, _lib.PROBE_FIELDS, stream_handle()))
    return {"sclk_mhz_under_load": out[0], "valu_f32_fma_T_lane_ops_s": out[1], "hbm_copy_GBs": out[2],
            "valu_kernel_ms": out[3], "copy_kernel_ms": out[4], "compute_units": int(out[5])}
