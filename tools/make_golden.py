"""Generate golden vectors by running the reference in the build container.

Writes small ``.npz`` fixtures into ``tests/golden/``.  The reference code is
imported from ``/root/reference`` (never copied); zero poses come from the
``.npz`` assets (decoded without unpickling).  Inputs are the deterministic
synthetic frames of ``rtg.synth`` (no recorded mocap ships with the reference).

Fixtures (all float32 unless noted):
  full_body_pos_precise.npz  VtrdynFullBodyPosRetargeter(precise_gripper=True)   512 frames
  full_body_pos_binary.npz   VtrdynFullBodyPosRetargeter(precise_gripper=False)  128 frames
  upper_body.npz             HuUpperBodyFromMocapRetarget                        512 frames
  full_body_rot.npz          VtrdynFullBodyRetargeter                            256 frames
  body_rot.npz               Mocap2HuBodyRetargeter                              256 frames
  kinematics.npz             cal_forward_kinematics / cal_local_rotation /
                             SkeletonState FK on hu_v5, vtrdyn, vtrdyn_full, noitom
  primitives.npz             per-primitive vectors incl. edge cases
  kat_rotation_test.npz      retarget/rotation_test.py known-answer test, restated
  zero_pose.npz              zero-pose global translations as the reference computes them
  main_retarget.npz          retarget/main.py retarget_from_global_translation end to end (48 frames)
  expmap.npz                 the rotation3d exp-map family (quat_to_exp_map ... quat_angle_axis) with edge cases
  full_body_pos_edge.npz     degenerate frames per solver (zero-length / axis-aligned arm segments, straight
  full_body_rot_edge.npz     elbows, near gimbal lock, collapsed / coplanar / mirrored hands, NaN / inf points,
  body_rot_edge.npz          zero and NaN quaternions): per frame the reference's outputs, or the exception it
  upper_body_edge.npz        raised (status 1 = RuntimeError from torch.linalg.svd, 2 = ValueError from scipy)
"""
from __future__ import annotations

import json
import os
import sys
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, HERE)

import refharness as rh  # noqa: E402

synth = rh.load_rtg_module("synth")

OUT = os.path.join(REPO, "tests", "golden")
warnings.filterwarnings("ignore")


def t2n(t):
    return t.detach().cpu().numpy().astype(np.float32).copy()


def gen_full_body_pos(ref, torch, precise, n, seed):
    full = rh.ref_zero_pose(ref, "vtrdyn_full")
    hu = rh.ref_zero_pose(ref, "hu_v5")
    s = ref.full_body_pos.VtrdynFullBodyPosRetargeter(full, hu, precise_gripper=precise)
    body, lh, rhd = synth.synth_full_body_inputs(n, seed)
    dof, lr, bg = [], [], []
    for i in range(n):
        a, b, c = s.retarget(torch.from_numpy(body[i]), torch.from_numpy(lh[i]), torch.from_numpy(rhd[i]))
        lr.append(t2n(a)); dof.append(t2n(b)); bg.append(t2n(c))
    bg = np.stack(bg)
    return dict(body=body, lh=lh, rh=rhd, dof=np.stack(dof), local_rot=np.stack(lr),
                body_rot_rows=bg[:, [10, 14, 39]], body_rot_untouched_identity=np.array(
                    np.all(np.delete(bg, [10, 14, 39], axis=1) == np.array([0, 0, 0, 1], np.float32))),
                precise_gripper=np.array(precise), seed=np.array(seed))


def gen_upper_body(ref, torch, n, seed):
    vz = rh.ref_zero_pose(ref, "vtrdyn")
    hu = rh.ref_zero_pose(ref, "hu_v5")
    s = ref.upper_body.HuUpperBodyFromMocapRetarget(vz, hu)
    x = synth.synth_upper_body_inputs(n, seed)
    dof, lr, kq = [], [], []
    zl = vz.local_translation
    for i in range(n):
        xt = torch.from_numpy(x[i])
        a, b = s.retarget_from_global_translation(xt)
        lr.append(t2n(a)); dof.append(t2n(b))
        st = ref.transform3d.coord_transform(xt, dir=torch.Tensor([-1, -1, 1]))
        kq.append(t2n(ref.transform3d.cal_joint_quat(zl[[17, 13, 11]].unsqueeze(0),
                                                     (st[[17, 13, 11]] - st[[10]]).unsqueeze(0))).reshape(4))
    return dict(x=x, dof=np.stack(dof), local_rot=np.stack(lr), kabsch_q=np.stack(kq), seed=np.array(seed))


def gen_full_body_rot(ref, torch, n, seed):
    full = rh.ref_zero_pose(ref, "vtrdyn_full")
    hu = rh.ref_zero_pose(ref, "hu_v5")
    s = ref.full_body.VtrdynFullBodyRetargeter(full, hu)
    brot, bpos, lh, rhd = synth.synth_full_body_rot_inputs(n, seed)
    dof, lr = [], []
    for i in range(n):
        a, b = s.retarget(torch.from_numpy(brot[i]), torch.from_numpy(bpos[i]), None, torch.from_numpy(lh[i]),
                          None, torch.from_numpy(rhd[i]))
        lr.append(t2n(a)); dof.append(t2n(b))
    return dict(body_rot=brot, body_pos=bpos, lh=lh, rh=rhd, dof=np.stack(dof), local_rot=np.stack(lr),
                seed=np.array(seed))


def gen_body_rot(ref, torch, n, seed):
    br_mod = rh.load_body_retargeter_module(ref)
    vz = rh.ref_zero_pose(ref, "vtrdyn")
    hu = rh.ref_zero_pose(ref, "hu_v5")
    s = br_mod.Mocap2HuBodyRetargeter(vz, hu)
    _, grot = synth.synth_body21_pose(n, seed)
    dof, lr = [], []
    for i in range(n):
        a, b = s.retarget_from_pose(torch.from_numpy(grot[i]))
        lr.append(t2n(a)); dof.append(t2n(b))
    return dict(global_rot=grot, dof=np.stack(dof), local_rot=np.stack(lr), seed=np.array(seed))


def gen_kinematics(ref, torch, n):
    out = {}
    for k, name in enumerate(["hu_v5", "vtrdyn", "vtrdyn_full", "noitom"]):
        st = rh.ref_skeleton_state(ref, name)
        tree = st.skeleton_tree
        J = tree.num_joints
        lr = synth.random_local_quats(n, J, 100 + k)
        rt = np.random.default_rng(200 + k).normal(0, 0.3, (n, 3)).astype(np.float32)
        gr, gp = ref.rkm.cal_forward_kinematics(torch.from_numpy(lr), torch.from_numpy(rt),
                                                tree.parent_indices, tree.local_translation)
        loc = ref.rkm.cal_local_rotation(gr, tree.parent_indices)
        sk = ref.skeleton3d.SkeletonState.from_rotation_and_root_translation(
            tree, torch.from_numpy(lr), torch.from_numpy(rt), is_local=True)
        out[f"{name}_local_rot"] = lr
        out[f"{name}_root_t"] = rt
        out[f"{name}_g_rot"] = t2n(gr)
        out[f"{name}_g_pos"] = t2n(gp)
        out[f"{name}_inv_local"] = t2n(loc)
        out[f"{name}_state_g_rot"] = t2n(sk.global_rotation)
        out[f"{name}_state_g_pos"] = t2n(sk.global_translation)
        skg = ref.skeleton3d.SkeletonState.from_rotation_and_root_translation(
            tree, torch.from_numpy(out[f"{name}_state_g_rot"]), torch.from_numpy(rt), is_local=False)
        out[f"{name}_state_local_rot"] = t2n(skg.local_rotation)
    return out


def gen_dof_fk(ref, torch, n):
    """HuForwardModel.forward_kinematics (robot_kinematics_model/hu_forward_model.py:17-33), evaluated step by
    step with the reference's own functions: the module itself imports motion_convert.*, which the reference
    does not ship.  hu (33 links, robot_config/Hu.py tables) with clip_angles=True and False; hu_v5 (31 links,
    Hu_v5 axes; its 32-entry limit tables cannot broadcast against 30 DOFs) without clipping."""
    import importlib
    out = {}
    cases = (("hu", "retarget.robot_config.Hu", True), ("hu", "retarget.robot_config.Hu", False),
             ("hu_v5", "retarget.robot_config.Hu_v5", False))
    for k, (name, mod, clip) in enumerate(cases):
        cfg = importlib.import_module(mod)
        tree = rh.ref_skeleton_state(ref, name).skeleton_tree
        J = tree.num_joints
        rng = np.random.default_rng(300 + k)
        ang = rng.uniform(-3.5, 3.5, (n, J - 1, 1)).astype(np.float32)   # well beyond the limits: clip is exercised
        ang[:4] = 0.0
        root_rot = _rand_quats(rng, n).reshape(n, 1, 4)
        root_t = rng.normal(0, 0.3, (n, 3)).astype(np.float32)
        a = torch.from_numpy(ang)
        if clip:   # HuForwardModel._clip_angles :27-33 (forward value of the straight-through form)
            lo = cfg.Hu_DOF_LOWER.reshape(1, -1, 1)
            hi = cfg.Hu_DOF_UPPER.reshape(1, -1, 1)
            c = torch.clamp(a.clone(), min=lo, max=hi)
            a = (c - a).detach() + a
        axis = torch.eye(3)[cfg.Hu_DOF_AXIS].repeat(n, 1, 1).clone()                 # :16, :21
        lr = ref.rotation3d.quat_from_angle_axis(a.reshape(-1), axis.reshape(-1, 3))  # :22
        lr = lr.reshape(n, J - 1, 4)
        lr = torch.concatenate([torch.from_numpy(root_rot), lr], dim=1)             # :24
        gr, gp = ref.rkm.cal_forward_kinematics(motion_local_rotation=lr, motion_root_translation=torch.from_numpy(root_t),
                                                parent_indices=tree.parent_indices,
                                                zero_pose_local_translation=tree.local_translation)
        tag = f"{name}_{'clip' if clip else 'noclip'}"
        out[f"{tag}_dof"] = ang[..., 0]
        out[f"{tag}_root_rot"] = root_rot[:, 0]
        out[f"{tag}_root_t"] = root_t
        out[f"{tag}_axis"] = np.asarray(cfg.Hu_DOF_AXIS, np.int32)
        if clip:
            out[f"{tag}_lower"] = t2n(cfg.Hu_DOF_LOWER)
            out[f"{tag}_upper"] = t2n(cfg.Hu_DOF_UPPER)
        out[f"{tag}_g_rot"] = t2n(gr)
        out[f"{tag}_g_pos"] = t2n(gp)
    return out


def gen_motion_prep(ref, torch, L=64):
    """retarget/main.py motion-level prep, called on the reference's own code:
    coord_transform (:170) -> Retarget.rescale_motion_to_standard_size (:37-47) ->
    RetargetHuV5fromMocap._rebuild_with_vtrdyn_zero_pose (:116-165, its SkeletonMotion's global rotations).
    Inputs: smooth synthetic VTRDyn body motion (21 joints, raw mocap frame).  Also quat_between_two_vecs
    (transform3d.py:8-21) on random pairs and on an all-degenerate batch (the batch-level identity branch)."""
    main = rh.load_main_module(ref)
    zp = rh.ref_zero_pose(ref, "vtrdyn")
    x = synth.synth_upper_body_inputs(L, 4242)                     # raw VTRDyn positions (B, 21, 3)
    g = np.random.default_rng(4243)                                  # other body sizes + marker jitter:
    x = (x * g.uniform(0.8, 1.25, (L, 1, 1)) + g.normal(0, 0.01, x.shape)).astype(np.float32)   # rescale has work
    xt = torch.from_numpy(x)
    m = ref.transform3d.coord_transform(xt, dir=torch.Tensor([-1, -1, 1]))
    rescaled = main.Retarget.rescale_motion_to_standard_size(m, zp)
    rt = main.RetargetHuV5fromMocap(zp, zp)
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):               # it prints the rebuild error
        motion = rt._rebuild_with_vtrdyn_zero_pose(rescaled)
    rng = np.random.default_rng(77)
    v1 = rng.normal(size=(512, 3)).astype(np.float32)
    v2 = rng.normal(size=(512, 3)).astype(np.float32)
    v2[:8] = -v1[:8]                                                 # antiparallel: real part 1 + dot ~ 0
    v2[8:16] = v1[8:16] * 3.0                                         # parallel
    qb = ref.transform3d.quat_between_two_vecs(torch.from_numpy(v1), torch.from_numpy(v2))
    qb0 = ref.transform3d.quat_between_two_vecs(torch.from_numpy(v1[:4]), torch.zeros(4, 3))
    return {"raw": x, "rescaled": t2n(rescaled), "g_rot": t2n(motion.global_rotation),
            "root_t": t2n(motion.root_translation), "qb_v1": v1, "qb_v2": v2, "qb": t2n(qb), "qb_zero": t2n(qb0)}


def gen_main_retarget(ref, torch, L=48):
    """retarget/main.py RetargetHuV5fromMocap.retarget_from_global_translation (:169-279), the reference's own
    code end to end: coord_transform -> rescale -> _rebuild_with_vtrdyn_zero_pose -> the per-frame arm maps on
    the rebuilt motion -> SkeletonState(is_local=True) -> SkeletonMotion(fps=30).  Its last call,
    plot_skeleton_H([mocap_motion, retargeted_motion]) (:280), is replaced by a capture of those two motions.
    The target is Hu v5 from its pickled zero pose (asset/hu/hu_v5.urdf is not shipped)."""
    main = rh.load_main_module(ref)
    zv = rh.ref_zero_pose(ref, "vtrdyn")
    hu = rh.ref_zero_pose(ref, "hu_v5")
    x = synth.synth_upper_body_inputs(L, 5151)
    g = np.random.default_rng(5152)
    x = (x * g.uniform(0.8, 1.25, (L, 1, 1)) + g.normal(0, 0.01, x.shape)).astype(np.float32)
    captured = []
    main.plot_skeleton_H = lambda motions, *a, **k: captured.extend(motions)
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):                  # it prints per-frame timings
        main.RetargetHuV5fromMocap(zv, hu).retarget_from_global_translation(torch.from_numpy(x))
    mocap, robot = captured
    return {"x": x, "mocap_g_rot": t2n(mocap.global_rotation), "mocap_g_pos": t2n(mocap.global_translation),
            "mocap_local_rot": t2n(mocap.local_rotation), "robot_local_rot": t2n(robot.local_rotation),
            "robot_g_rot": t2n(robot.global_rotation), "robot_g_pos": t2n(robot.global_translation),
            "robot_velocity": t2n(robot.global_velocity), "robot_angular_velocity": t2n(robot.global_angular_velocity),
            "fps": np.array(robot.fps)}


def _rand_quats(rng, n):
    q = rng.normal(size=(n, 4))
    q /= np.linalg.norm(q, axis=-1, keepdims=True)
    return q.astype(np.float32)


def gen_motion(ref, torch, L=96):
    """SkeletonMotion.from_skeleton_state (skeleton3d.py:1026-1049): smooth random Hu motion at 30 fps."""
    st0 = rh.ref_skeleton_state(ref, "hu_v5")
    tree = st0.skeleton_tree
    J = tree.num_joints
    rng = np.random.default_rng(77)
    # smooth trajectories: cumulative small axis-angle steps per joint
    steps = rng.normal(0, 0.05, (L, J, 3)).cumsum(0)
    ang = np.linalg.norm(steps, axis=-1, keepdims=True)
    q = np.concatenate([steps / np.maximum(ang, 1e-12) * np.sin(ang / 2), np.cos(ang / 2)], -1).astype(np.float32)
    rt = (rng.normal(0, 0.01, (L, 3)).cumsum(0)).astype(np.float32)
    st = ref.skeleton3d.SkeletonState.from_rotation_and_root_translation(tree, torch.from_numpy(q), torch.from_numpy(rt),
                                                                         is_local=True)
    mo = ref.skeleton3d.SkeletonMotion.from_skeleton_state(st, fps=30)
    return dict(local_rot=q, root_t=rt, global_rot=t2n(st.global_rotation), global_pos=t2n(st.global_translation),
                global_velocity=t2n(mo.global_velocity), global_angular_velocity=t2n(mo.global_angular_velocity),
                tensor=t2n(mo.tensor), fps=np.array(30))


def gen_primitives(ref, torch):
    r3 = ref.rotation3d
    tf = ref.transform3d
    fb = ref.full_body_pos
    rng = np.random.default_rng(7)
    out = {}
    n = 1024
    a = _rand_quats(rng, n) * rng.uniform(0.5, 2.0, (n, 1)).astype(np.float32)
    b = _rand_quats(rng, n)
    out["qm_a"], out["qm_b"] = a, b
    out["quat_mul"] = t2n(r3.quat_mul(torch.from_numpy(a), torch.from_numpy(b)))
    out["quat_mul_norm"] = t2n(r3.quat_mul_norm(torch.from_numpy(a), torch.from_numpy(b)))
    out["quat_normalize"] = t2n(r3.quat_normalize(torch.from_numpy(a)))
    v = rng.normal(size=(n, 3)).astype(np.float32)
    out["qr_v"] = v
    out["quat_rotate"] = t2n(r3.quat_rotate(torch.from_numpy(b), torch.from_numpy(v)))
    # quat_from_angle_axis: random + small / pi / >pi / deadzone angles
    ang = np.concatenate([rng.uniform(-4, 4, n - 16),
                          np.array([0, 1e-4, -1e-4, 3e-4, 4.9e-4, 6e-4, -6e-4, np.pi, -np.pi, 2 * np.pi,
                                    3.5, -3.5, 1e-7, 0.5, -0.5, 1.0])]).astype(np.float32)
    axs = rng.normal(size=(n, 3)).astype(np.float32)
    axs[-16:] = np.eye(3, dtype=np.float32)[np.arange(16) % 3]
    out["qaa_angle"], out["qaa_axis"] = ang, axs
    out["quat_from_angle_axis"] = t2n(r3.quat_from_angle_axis(torch.from_numpy(ang), torch.from_numpy(axs)))
    # quat_from_rotation_matrix: random rotations + 180deg + tie cases
    from scipy.spatial.transform import Rotation as sRot
    mats = sRot.from_quat(_rand_quats(rng, n - 8).astype(np.float64)).as_matrix()
    special = [np.diag([1.0, -1, -1]), np.diag([-1.0, 1, -1]), np.diag([-1.0, -1, 1]), np.eye(3),
               sRot.from_rotvec([np.pi / 2, 0, 0]).as_matrix(), sRot.from_rotvec([0, np.pi / 2, 0]).as_matrix(),
               sRot.from_rotvec([0, 0, np.pi / 2]).as_matrix(), sRot.from_rotvec([np.pi / 2, np.pi / 2, 0]).as_matrix()]
    mats = np.concatenate([mats, np.stack(special)]).astype(np.float32)
    out["qrm_m"] = mats
    out["quat_from_rotation_matrix"] = t2n(r3.quat_from_rotation_matrix(torch.from_numpy(mats)))
    # quat_to_dof_pos on (30,4) chunks -- the hot-path shape (atan2 takes glibc's scalar path)
    q31 = _rand_quats(rng, 64 * 31).reshape(64, 31, 4)
    q31[..., 3] = np.abs(q31[..., 3])
    small = np.array([0, 1e-4, 3e-4, 4.9e-4, 6e-4, 1e-3, 1e-2, 3.1], np.float32)
    for i, s in enumerate(small):   # single-axis small rotations (exp-map deadzone)
        q31[i, 1:, :] = 0
        q31[i, 1:, 3] = np.cos(s / 2)
        q31[i, 1:, 1] = np.sin(s / 2)
    q31 = q31.astype(np.float32)
    out["dof_q31"] = q31
    out["quat_to_dof_pos"] = np.stack([t2n(tf.quat_to_dof_pos(torch.from_numpy(q31[i, 1:]), ref.Hu_v5.Hu_DOF_AXIS))
                                       for i in range(len(q31))])
    # radians_between_vecs / proj_in_plane (1-D only in the reference)
    m = 512
    v1 = rng.normal(size=(m, 3)).astype(np.float32)
    v2 = rng.normal(size=(m, 3)).astype(np.float32)
    v2[:8] = v1[:8] * np.float32(2.0)                       # parallel: sign(0) -> 0
    v2[8:16] = v1[8:16] + rng.normal(0, 1e-4, (8, 3)).astype(np.float32)   # near parallel
    nn = rng.normal(size=(m, 3)).astype(np.float32)
    out["rbv_v1"], out["rbv_v2"], out["rbv_n"] = v1, v2, nn
    out["radians_between_vecs"] = np.array([tf.radians_between_vecs(torch.from_numpy(v1[i]), torch.from_numpy(v2[i]),
                                                                    torch.from_numpy(nn[i])).item()
                                            for i in range(m)], np.float32)
    eye = torch.eye(3)
    out["proj_in_plane_y"] = np.stack([t2n(tf.proj_in_plane(torch.from_numpy(v1[i]), eye[1])) for i in range(m)])
    out["proj_in_plane_z"] = np.stack([t2n(tf.proj_in_plane(torch.from_numpy(v1[i]), eye[2])) for i in range(m)])
    # cal_joint_quat (Kabsch) with 3 and 5 points
    for npts in (3, 5):
        k = 256
        Z = rng.normal(0, 0.1, (k, npts, 3)).astype(np.float32)
        if npts == 3:
            Z[:k // 2, :, 0] = 0.0          # rank-2 like the torso fit
        R = sRot.from_quat(_rand_quats(rng, k).astype(np.float64)).as_matrix()
        M = (np.einsum("kij,knj->kni", R, Z.astype(np.float64)) + rng.normal(0, 0.002, Z.shape)).astype(np.float32)
        M[-4:] = -M[-4:]                     # reflection-only fits (det fix path)
        out[f"cjq{npts}_Z"], out[f"cjq{npts}_M"] = Z, M
        out[f"cal_joint_quat{npts}"] = np.stack([t2n(tf.cal_joint_quat(torch.from_numpy(Z[i:i + 1]),
                                                                       torch.from_numpy(M[i:i + 1]))).reshape(4)
                                                 for i in range(k)])
    # quat_in_xyz_axis (scipy float64 Euler) incl. gimbal lock
    qe = _rand_quats(rng, 512)
    gl = sRot.from_euler("XYZ", [[0.3, np.pi / 2, 0.2], [0.1, -np.pi / 2, -0.4]]).as_quat().astype(np.float32)
    qe[:2] = gl
    out["qxyz_q"] = qe
    for seq in ("XYZ", "YXZ", "ZYX"):
        res = [tf.quat_in_xyz_axis(torch.from_numpy(qe[i:i + 1]), seq) for i in range(len(qe))]
        out[f"quat_in_xyz_axis_{seq}"] = np.stack([np.stack([t2n(r[j]).reshape(4) for j in range(3)]) for r in res])
    # cal_shoulderPR / cal_elbowP_and_shoulderY
    k = 512
    sv1 = rng.normal(0, 0.3, (k, 3)).astype(np.float32)
    par = _rand_quats(rng, k)
    par[:, 3] = np.abs(par[:, 3])
    full = rh.ref_zero_pose(ref, "vtrdyn_full")
    sv0 = np.broadcast_to(t2n(full.local_translation[13]), (k, 3)).copy()
    ev0 = np.broadcast_to(t2n(full.local_translation[14]), (k, 3)).copy()
    out["sh_v1"], out["sh_v0"], out["el_v0"], out["sh_parent"] = sv1, sv0, ev0, par
    spr, epy = [], []
    for i in range(k):
        p_, r_ = fb.cal_shoulderPR(torch.from_numpy(sv1[i]), torch.from_numpy(sv0[i]), torch.from_numpy(par[i:i + 1]))
        spr.append(np.stack([t2n(p_).reshape(4), t2n(r_).reshape(4)]))
        y_, e_ = fb.cal_elbowP_and_shoulderY(torch.from_numpy(sv1[i]), torch.from_numpy(ev0[i]),
                                             torch.from_numpy(par[i:i + 1]))
        epy.append(np.stack([t2n(y_).reshape(4), t2n(e_).reshape(4)]))
    out["cal_shoulderPR"] = np.stack(spr)
    out["cal_elbowP_and_shoulderY"] = np.stack(epy)
    return out


def gen_expmap(ref, torch):
    """quat_to_exp_map / quat_to_angle_axis / normalize_angle / quat_abs / quat_unit / quat_angle_axis
    (rotation3d.py:41-56, 230-240, 582-627), called on chunks of 16 like the reference's per-frame use (torch
    takes glibc's scalar atan2f below 32 elements).  Edge cases: w < 0, w = +-1, the 1e-5 sin_theta deadzone,
    the angle table's w = 0.25 boundary, angles at +-pi, zero / tiny quaternions."""
    r3 = ref.rotation3d
    rng = np.random.default_rng(17)
    n = 2048
    q = _rand_quats(rng, n)
    q[: n // 4] *= -1.0                                             # w < 0
    w_edge = np.float32([1.0, -1.0, 0.0, 0.25, np.nextafter(np.float32(0.25), np.float32(0)),
                         np.nextafter(np.float32(0.25), np.float32(1)), np.float32(1) - np.float32(2 ** -24),
                         np.float32(1) - np.float32(2 ** -23), 0.9999999, 0.99999994, 1 - 5e-11, 1 - 1e-10,
                         0.5, -0.5, 0.70710677, 0.9999, 0.999999])
    m = len(w_edge)
    ax = rng.standard_normal((m, 3)).astype(np.float32)
    ax /= np.linalg.norm(ax, axis=1, keepdims=True)
    s = np.sqrt(np.maximum(0.0, 1.0 - w_edge.astype(np.float64) ** 2)).astype(np.float32)
    q[n // 4: n // 4 + m] = np.concatenate([ax * s[:, None], w_edge[:, None]], 1)
    tiny = rng.standard_normal((64, 3)).astype(np.float32) * np.float32(3e-6)    # |xyz| around the deadzone
    q[n // 2: n // 2 + 64] = np.concatenate([tiny, np.sqrt(1 - (tiny ** 2).sum(1, keepdims=True))], 1)
    out = {"em_q": q}
    chunks = [torch.from_numpy(q[i:i + 16]) for i in range(0, n, 16)]
    out["quat_to_exp_map"] = np.concatenate([t2n(r3.quat_to_exp_map(c)) for c in chunks])
    aa = [r3.quat_to_angle_axis(c) for c in chunks]
    out["quat_to_angle_axis"] = np.concatenate([np.concatenate([t2n(a)[:, None], t2n(x)], 1) for a, x in aa])
    x = np.concatenate([rng.uniform(-10, 10, 1536), np.float32([0.0, -0.0, np.pi, -np.pi, 2 * np.pi, 3 * np.pi,
                                                                1e-7, -1e-7, 7.0, -7.0])]).astype(np.float32)
    x = np.concatenate([x, rng.uniform(-10, 10, (-len(x)) % 16).astype(np.float32)])
    out["na_x"] = x
    out["normalize_angle"] = np.concatenate([t2n(r3.normalize_angle(torch.from_numpy(x[i:i + 16])))
                                             for i in range(0, len(x), 16)])
    g = _rand_quats(rng, 512) * rng.uniform(1e-3, 3.0, (512, 1)).astype(np.float32)
    g[:4] = 0.0
    g[4:8] *= np.float32(1e-10)                                     # below the 1e-9 clamp
    out["qa_q"] = g
    out["quat_abs"] = np.concatenate([t2n(r3.quat_abs(torch.from_numpy(g[i:i + 16]))) for i in range(0, 512, 16)])
    out["quat_unit"] = np.concatenate([t2n(r3.quat_unit(torch.from_numpy(g[i:i + 16]))) for i in range(0, 512, 16)])
    u = _rand_quats(rng, 512)
    u[:2] = np.float32([[0, 0, 0, 1], [0, 0, 0, -1]])
    out["qaa_q"] = u
    res = []
    for i in range(0, 512, 16):
        a, xyz = r3.quat_angle_axis(torch.from_numpy(u[i:i + 16].copy()))   # the reference divides in place
        res.append(np.concatenate([t2n(a)[:, None], t2n(xyz)], 1))
    out["quat_angle_axis"] = np.concatenate(res)
    return out


def gen_overlay_extras(ref, torch):
    """The rest of the rotation3d / transform3d surface the drop-in now exports (rotation3d.py:101-108, 243-261,
    338-350, 398-427, 465-473, 479-556, 629-661; transform3d.py:8-21, 146-174), called on chunks of 16 like the
    per-frame callers (torch takes glibc's scalar atan2f below 32 elements).  Edge cases: zero / tiny / > pi
    exp-maps, slerp with cos < 0, t in {0, 1}, nearly equal and identical quaternions, parallel and opposite vectors."""
    r3, t3 = ref.rotation3d, ref.transform3d
    rng = np.random.default_rng(29)
    out = {}
    n = 1024
    e = (rng.standard_normal((n, 3)) * rng.uniform(0, 4, (n, 1))).astype(np.float32)
    e[:8] = 0.0
    e[8:16] *= np.float32(1e-6)
    e[16:24] = rng.standard_normal((8, 3)).astype(np.float32) * np.float32(3e-6)
    e[24:32] *= np.float32(3.0)                                   # |e| > pi: normalize_angle wraps
    out["em_e"] = e
    chunks = [torch.from_numpy(e[i:i + 16]) for i in range(0, n, 16)]
    aa = [r3.exp_map_to_angle_axis(c) for c in chunks]
    out["exp_map_to_angle_axis"] = np.concatenate([np.concatenate([t2n(a)[:, None], t2n(x)], 1) for a, x in aa])
    out["exp_map_to_quat"] = np.concatenate([t2n(r3.exp_map_to_quat(c)) for c in chunks])
    out["t3_exp_map_to_quat"] = np.concatenate([t2n(t3.exp_map_to_quat(c)) for c in chunks])
    q0, q1 = _rand_quats(rng, n), _rand_quats(rng, n)
    q1[: n // 4] *= -1.0                                          # cos(half) < 0: the shortest-arc flip
    q1[n // 4: n // 4 + 16] = q0[n // 4: n // 4 + 16]              # identical: |cos| >= 1
    q1[n // 4 + 16: n // 4 + 32] = (q0[n // 4 + 16: n // 4 + 32] + np.float32(1e-4)).astype(np.float32)
    t = rng.uniform(0, 1, (n, 1)).astype(np.float32)
    t[:4] = 0.0
    t[4:8] = 1.0
    out["sl_q0"], out["sl_q1"], out["sl_t"] = q0, q1, t
    out["quat_slerp"] = np.concatenate([t2n(t3.quat_slerp(torch.from_numpy(q0[i:i + 16]), torch.from_numpy(q1[i:i + 16]),
                                                          torch.from_numpy(t[i:i + 16]))) for i in range(0, n, 16)])
    v1 = rng.standard_normal((n, 3)).astype(np.float32)
    v2 = rng.standard_normal((n, 3)).astype(np.float32)
    v2[:8] = v1[:8] * np.float32(2.0)                            # parallel
    v2[8:16] = -v1[8:16]                                          # opposite
    out["qb_v1"], out["qb_v2"] = v1, v2
    out["quat_between_two_vecs"] = np.concatenate([t2n(t3.quat_between_two_vecs(torch.from_numpy(v1[i:i + 16]),
                                                                                torch.from_numpy(v2[i:i + 16])))
                                                   for i in range(0, n, 16)])
    xyz = (rng.standard_normal((64, 3)) * 0.3).astype(np.float32)
    xyz /= np.maximum(1.0, np.linalg.norm(xyz, axis=1, keepdims=True) * 1.01).astype(np.float32)
    out["qx_xyz"] = xyz
    out["quat_from_xyz"] = np.stack([t2n(r3.quat_from_xyz(torch.from_numpy(x.copy()))) for x in xyz])
    q = _rand_quats(rng, n)
    q[: n // 2] *= rng.uniform(0.5, 2.0, (n // 2, 1)).astype(np.float32)   # not unit: rot_matrix_from_quaternion's 2/|q|^2
    out["pq_q"] = q
    qc = [torch.from_numpy(q[i:i + 16]) for i in range(0, n, 16)]
    out["rot_matrix_from_quaternion"] = np.concatenate([t2n(r3.rot_matrix_from_quaternion(c)) for c in qc])
    m = rng.standard_normal((n, 3, 3)).astype(np.float32)
    out["det_m"] = m
    out["rot_matrix_det"] = np.concatenate([t2n(r3.rot_matrix_det(torch.from_numpy(m[i:i + 16]))) for i in range(0, n, 16)])
    for k in ("x", "y", "z", "xy", "xz"):
        out[f"project_quat_to_axis_{k}"] = np.concatenate([t2n(getattr(r3, f"project_quat_to_axis_{k}")(c)) for c in qc])
    for ax in range(3):
        out[f"extract_rotation_along_axis_{ax}"] = np.concatenate([t2n(r3.extract_rotation_along_axis(c, ax)) for c in qc])
    for z_up in (True, False):
        out[f"quat_yaw_rotation_{int(z_up)}"] = np.concatenate([t2n(r3.quat_yaw_rotation(c, z_up)) for c in qc])
    out["quat_to_eular"] = np.stack([r3.quat_to_eular(torch.from_numpy(x.copy())) for x in q[:256]]).astype(np.float64)
    eu = np.zeros((64, 4, 4), np.float32)
    for i in range(64):
        eu[i, :3, :3] = rng.standard_normal((3, 3))
        eu[i, :3, 3] = rng.standard_normal(3)
        eu[i, 3, 3] = 1.0
    out["eu_m"] = eu
    out["euclidean_to_transform"] = t2n(r3.euclidean_to_transform(torch.from_numpy(eu)))
    return out


# ---------------------------------------------------------------------------------------------------------------
# Degenerate frames (VERDICT r03 "What's weak" #1).  The reference solves one frame per call and raises on some of
# these: torch.linalg.svd on a NaN Kabsch matrix (transform3d.py:40, RuntimeError) and scipy from_quat on a zero /
# NaN quaternion (transform3d.py:53, ValueError).  Each fixture records, per frame, the outputs or the exception.
# ---------------------------------------------------------------------------------------------------------------
STATUS_OK, STATUS_SVD, STATUS_ZERO_NORM = 0, 1, 2   # include/rtg.h rtg_frame_error


def classify(e: BaseException) -> int:
    msg = str(e)
    if isinstance(e, ValueError) and "zero norm quaternions" in msg:
        return STATUS_ZERO_NORM
    if isinstance(e, RuntimeError) and "linalg.svd" in msg and "non-finite values" in msg:
        return STATUS_SVD
    raise AssertionError(f"unexpected exception from the reference: {type(e).__name__}: {msg}")


def _rot_about(points, center, axis, angle):
    """Rotate points (n,3) about `center` by `angle` around the unit `axis` (float64 Rodrigues), float32 out."""
    from scipy.spatial.transform import Rotation as sRot
    R = sRot.from_rotvec(np.asarray(axis, np.float64) * angle).as_matrix()
    return ((points.astype(np.float64) - center) @ R.T + center).astype(np.float32)


def edge_full_body_frames():
    """~64 degenerate VtrdynFullBodyPosRetargeter frames: edits of the VTRDYN_FULL zero pose (whose torso and arm
    frames are the identity, so "along y" is along the shoulder plane's normal) and of 8 random synthetic poses."""
    zp = np.load(os.path.join(OUT, "zero_pose.npz"))
    zg = zp["vtrdyn_full_global_t"]
    base = [(zg[synth.FULL_TO_BODY].copy(), zg[synth.LH_SLICE].copy(), zg[synth.RH_SLICE].copy())]
    rb, rl, rr = synth.synth_full_body_inputs(8, 97)
    base += [(rb[i].copy(), rl[i].copy(), rr[i].copy()) for i in range(8)]
    frames, names = [], []

    def add(name, b, l, r):
        frames.append((b, l, r))
        names.append(name)

    f32 = np.float32
    b0, l0, r0 = base[0]
    add("zero pose", b0, l0, r0)
    for k, (bb, ll, rr_) in enumerate(base):
        tag = "zero" if k == 0 else f"rand{k}"
        b = bb.copy(); b[19] = b[18]; add(f"{tag}: zero-length left upper arm", b, ll, rr_)
        b = bb.copy(); b[16] = b[15]; add(f"{tag}: zero-length right forearm", b, ll, rr_)
        b = bb.copy(); b[20] = b[19] + (b[19] - b[18]); add(f"{tag}: straight left elbow", b, ll, rr_)
        l = ll.copy(); l[:] = l[0]; add(f"{tag}: collapsed left hand", bb, l, rr_)
        b = bb.copy(); b[13, 2] = np.nan; add(f"{tag}: NaN torso point", b, ll, rr_)
        r = rr_.copy(); r[6, 0] = np.nan; add(f"{tag}: NaN right Kabsch hand point", bb, ll, r)
    # the zero pose: arm segments along the plane normals (their projections vanish)
    for side, (sh, el, wr) in (("left", (18, 19, 20)), ("right", (14, 15, 16))):
        b = b0.copy(); b[el] = b[sh] + f32([0, 0.3, 0]); b[wr] = b[el] + f32([0.25, 0, 0])
        add(f"zero: {side} upper arm along y", b, l0, r0)
        b = b0.copy(); b[el] = b[sh] + f32([0, 0, 0.3]); b[wr] = b[el] + f32([0.25, 0, 0])
        add(f"zero: {side} upper arm along z", b, l0, r0)
        b = b0.copy(); b[el] = b[sh] + f32([0.3, 0, 0]); b[wr] = b[el] + f32([0, 0, 0.25])
        add(f"zero: {side} forearm along z", b, l0, r0)
        b = b0.copy(); b[wr] = b[el]; add(f"zero: {side} zero-length forearm", b, l0, r0)
    for sgn in (1, -1):   # the left hand pitched by +-90 degrees about the wrist: near the Euler split's gimbal lock
        l = _rot_about(l0, l0[0].astype(np.float64), [0, 1, 0], sgn * np.pi / 2)
        add(f"zero: left wrist pitched {'+' if sgn > 0 else '-'}90", b0, l, r0)
    l = l0.copy(); l[:, 2] = l[0, 2]; add("zero: coplanar left hand", b0, l, r0)
    l = l0.copy(); l[:, 0] = 2 * l[0, 0] - l[:, 0]; add("zero: mirrored left hand", b0, l, r0)
    l = l0.copy(); l[4, 1] = np.nan; add("zero: NaN left fingertip (gripper only)", b0, l, r0)
    l = l0.copy(); l[2, 1] = np.nan; add("zero: NaN left Kabsch hand point", b0, l, r0)
    b = b0.copy(); b[19, 0] = np.nan; add("zero: NaN left elbow", b, l0, r0)
    b = b0.copy(); b[17, 0] = np.inf; add("zero: inf torso point (inf * 0 = NaN in the Kabsch matrix)", b, l0, r0)
    b = b0.copy(); b[19, 0] = np.inf; add("zero: inf left elbow", b, l0, r0)
    b = b0.copy(); b[[17, 13, 11]] = b[10]; add("zero: collapsed torso", b, l0, r0)
    add("all-zero frame", np.zeros_like(b0), np.zeros_like(l0), np.zeros_like(r0))
    body = np.stack([f[0] for f in frames]).astype(np.float32)
    lh = np.stack([f[1] for f in frames]).astype(np.float32)
    rh = np.stack([f[2] for f in frames]).astype(np.float32)
    return body, lh, rh, names


def _run_frames(call, n, shapes):
    """Call the reference per frame; outputs (NaN where it raised), status, message."""
    outs = [np.full((n,) + sh, np.nan, np.float32) for sh in shapes]
    status = np.zeros(n, np.int8)
    msgs = []
    for i in range(n):
        try:
            res = call(i)
            for o, r in zip(outs, res):
                o[i] = t2n(r).reshape(o.shape[1:])
            msgs.append("")
        except Exception as e:  # noqa: BLE001 -- classified: only the two documented raises are accepted
            status[i] = classify(e)
            msgs.append(f"{type(e).__name__}: {str(e).strip().splitlines()[-1]}")
    return outs, status, np.array(msgs)


def gen_full_body_pos_edge(ref, torch):
    full = rh.ref_zero_pose(ref, "vtrdyn_full")
    hu = rh.ref_zero_pose(ref, "hu_v5")
    body, lh, rhd, names = edge_full_body_frames()
    out = dict(body=body, lh=lh, rh=rhd, names=np.array(names))
    for precise in (True, False):
        s = ref.full_body_pos.VtrdynFullBodyPosRetargeter(full, hu, precise_gripper=precise)
        (lr, dof, bg), status, msgs = _run_frames(
            lambda i: s.retarget(torch.from_numpy(body[i]), torch.from_numpy(lh[i]), torch.from_numpy(rhd[i])),
            len(body), [(31, 4), (30,), (59, 4)])
        tag = "precise" if precise else "binary"
        out.update({f"{tag}_dof": dof, f"{tag}_local_rot": lr, f"{tag}_body_rot": bg, f"{tag}_status": status,
                    f"{tag}_message": msgs, f"{tag}_recorded": np.array(len(s._motion_dof_pos))})
    return out


def gen_upper_body_edge(ref, torch):
    vz = rh.ref_zero_pose(ref, "vtrdyn")
    hu = rh.ref_zero_pose(ref, "hu_v5")
    s = ref.upper_body.HuUpperBodyFromMocapRetarget(vz, hu)
    x0 = synth.synth_upper_body_inputs(4, 88)
    frames, names = [], []
    for k in range(4):
        xx = x0[k].copy(); frames.append(xx); names.append(f"rand{k}")
        xx = x0[k].copy(); xx[19] = xx[18]; frames.append(xx); names.append(f"rand{k}: zero-length left upper arm")
        xx = x0[k].copy(); xx[16] = xx[15]; frames.append(xx); names.append(f"rand{k}: zero-length right forearm")
        xx = x0[k].copy(); xx[13, 1] = np.nan; frames.append(xx); names.append(f"rand{k}: NaN torso point")
        xx = x0[k].copy(); xx[20, 1] = np.nan; frames.append(xx); names.append(f"rand{k}: NaN left wrist")
        xx = x0[k].copy(); xx[[17, 13, 11]] = xx[10]; frames.append(xx); names.append(f"rand{k}: collapsed torso")
    x = np.stack(frames).astype(np.float32)
    (lr, dof), status, msgs = _run_frames(lambda i: s.retarget_from_global_translation(torch.from_numpy(x[i])),
                                          len(x), [(31, 4), (30,)])
    return dict(x=x, names=np.array(names), dof=dof, local_rot=lr, status=status, message=msgs)


def gen_full_body_rot_edge(ref, torch):
    full = rh.ref_zero_pose(ref, "vtrdyn_full")
    hu = rh.ref_zero_pose(ref, "hu_v5")
    s = ref.full_body.VtrdynFullBodyRetargeter(full, hu)
    brot, bpos, lh, rhd = synth.synth_full_body_rot_inputs(6, 99)
    frames, names = [], []

    def add(name, q, p, l, r):
        frames.append((q, p, l, r))
        names.append(name)

    for k in range(6):
        q, p, l, r = brot[k].copy(), bpos[k].copy(), lh[k].copy(), rhd[k].copy()
        add(f"rand{k}", q, p, l, r)
        pp = p.copy(); pp[19] = pp[18]; add(f"rand{k}: zero-length left upper arm", q, pp, l, r)
        pp = p.copy(); pp[16] = pp[15]; add(f"rand{k}: zero-length right forearm", q, pp, l, r)
        qq = q.copy(); qq[20] = 0; add(f"rand{k}: zero left wrist rotation", qq, p, l, r)
        qq = q.copy(); qq[13, 0] = np.nan; add(f"rand{k}: NaN right shoulder parent rotation", qq, p, l, r)
        ll = l.copy(); ll[7, 0] = np.nan; add(f"rand{k}: NaN left fingertip (gripper only)", q, p, ll, r)
    q = np.stack([f[0] for f in frames]).astype(np.float32)
    p = np.stack([f[1] for f in frames]).astype(np.float32)
    l = np.stack([f[2] for f in frames]).astype(np.float32)
    r = np.stack([f[3] for f in frames]).astype(np.float32)
    (lr, dof), status, msgs = _run_frames(
        lambda i: s.retarget(torch.from_numpy(q[i]), torch.from_numpy(p[i]), None, torch.from_numpy(l[i]), None,
                             torch.from_numpy(r[i])), len(q), [(31, 4), (30,)])
    return dict(body_rot=q, body_pos=p, lh=l, rh=r, names=np.array(names), dof=dof, local_rot=lr, status=status,
                message=msgs)


def gen_body_rot_edge(ref, torch):
    br_mod = rh.load_body_retargeter_module(ref)
    vz = rh.ref_zero_pose(ref, "vtrdyn")
    hu = rh.ref_zero_pose(ref, "hu_v5")
    s = br_mod.Mocap2HuBodyRetargeter(vz, hu)
    _, grot = synth.synth_body21_pose(6, 98)
    par = vz.parent_indices.numpy()
    frames, names = [], []
    for k in range(6):
        g = grot[k].copy(); frames.append(g); names.append(f"rand{k}")
        g = grot[k].copy(); g[18] = 0; frames.append(g); names.append(f"rand{k}: zero left shoulder rotation")
        g = grot[k].copy(); g[int(par[15])] = 0; frames.append(g); names.append(f"rand{k}: zero right elbow parent")
        g = grot[k].copy(); g[19, 2] = np.nan; frames.append(g); names.append(f"rand{k}: NaN left elbow rotation")
        g = grot[k].copy(); g[5] = 0; frames.append(g); names.append(f"rand{k}: zero rotation of an unused joint")
        g = grot[k].copy(); g[14] = -g[14]; frames.append(g); names.append(f"rand{k}: negated right shoulder")
    g = np.stack(frames).astype(np.float32)
    (lr, dof), status, msgs = _run_frames(lambda i: s.retarget_from_pose(torch.from_numpy(g[i])), len(g),
                                          [(31, 4), (30,)])
    return dict(global_rot=g, names=np.array(names), dof=dof, local_rot=lr, status=status, message=msgs)


def gen_kat(ref, torch):
    """retarget/rotation_test.py:95-152 restated as data: arm segments from known joint angles."""
    r3 = ref.rotation3d
    fb = ref.full_body_pos
    p = [torch.tensor([[0., 0., 0.]]), torch.tensor([[0., -1., 0.]]), torch.tensor([[0., -1., -1.]]),
         torch.tensor([[1., -1., -1.]])]
    vec0, vec1, vec2 = p[1] - p[0], p[2] - p[1], p[3] - p[2]
    f = torch.float32
    quat0 = r3.quat_from_angle_axis(torch.tensor([0.0], dtype=f), torch.tensor([0, 0, 1], dtype=f))
    q11 = r3.quat_from_angle_axis(torch.tensor([0.0], dtype=f), torch.tensor([0, 1, 0], dtype=f))
    q12 = r3.quat_from_angle_axis(torch.tensor([-0.0], dtype=f), torch.tensor([1, 0, 0], dtype=f))
    q13 = r3.quat_from_angle_axis(torch.tensor([-torch.pi / 6], dtype=f), torch.tensor([0, 0, 1], dtype=f))
    q2 = r3.quat_from_angle_axis(torch.tensor([torch.pi / 4], dtype=f), torch.tensor([0, 1, 0], dtype=f))
    q1 = r3.quat_mul_three(q11, q12, q13)
    v1t = r3.quat_rotate(r3.quat_mul_norm(quat0, q1), vec1)
    v2t = r3.quat_rotate(r3.quat_mul_norm(r3.quat_mul_norm(quat0, q1), q2), vec2)
    pitch, roll = fb.cal_shoulderPR(v1t[0], vec1[0], quat0)
    comb = r3.quat_mul_three(quat0, pitch, roll)
    v1cal = r3.quat_rotate(comb, vec1)
    yaw, elbow = fb.cal_elbowP_and_shoulderY(v2t[0], vec2[0], comb)
    v2cal = r3.quat_rotate(r3.quat_mul_three(comb, yaw, elbow), vec2)
    assert torch.allclose(v1cal, v1t, rtol=1e-3, atol=1e-6)
    assert torch.allclose(v2cal, v2t, rtol=1e-3, atol=1e-6)
    return dict(vec1=t2n(vec1), vec2=t2n(vec2), quat0=t2n(quat0), v1t=t2n(v1t), v2t=t2n(v2t),
                pitch=t2n(pitch), roll=t2n(roll), yaw=t2n(yaw), elbow=t2n(elbow), v1cal=t2n(v1cal), v2cal=t2n(v2cal))


def main() -> None:
    import torch
    torch.set_num_threads(1)
    ref = rh.load_reference()
    os.makedirs(OUT, exist_ok=True)
    zp = {}
    for name in ["hu_v5", "vtrdyn", "vtrdyn_full", "noitom", "hu"]:
        z = rh.ref_zero_pose(ref, name)
        zp[f"{name}_local_t"] = t2n(z.local_translation)
        zp[f"{name}_global_t"] = t2n(z.global_translation)
    np.savez_compressed(os.path.join(OUT, "zero_pose.npz"), **zp)
    jobs = {
        "full_body_pos_precise": lambda: gen_full_body_pos(ref, torch, True, 512, 1234),
        "full_body_pos_binary": lambda: gen_full_body_pos(ref, torch, False, 128, 4321),
        "upper_body": lambda: gen_upper_body(ref, torch, 512, 2345),
        "full_body_rot": lambda: gen_full_body_rot(ref, torch, 256, 3456),
        "body_rot": lambda: gen_body_rot(ref, torch, 256, 5678),
        "kinematics": lambda: gen_kinematics(ref, torch, 128),
        "primitives": lambda: gen_primitives(ref, torch),
        "motion": lambda: gen_motion(ref, torch),
        "kat_rotation_test": lambda: gen_kat(ref, torch),
        "dof_fk": lambda: gen_dof_fk(ref, torch, 128),
        "motion_prep": lambda: gen_motion_prep(ref, torch),
        "expmap": lambda: gen_expmap(ref, torch),
        "main_retarget": lambda: gen_main_retarget(ref, torch),
        "overlay_extras": lambda: gen_overlay_extras(ref, torch),
        "full_body_pos_edge": lambda: gen_full_body_pos_edge(ref, torch),
        "upper_body_edge": lambda: gen_upper_body_edge(ref, torch),
        "full_body_rot_edge": lambda: gen_full_body_rot_edge(ref, torch),
        "body_rot_edge": lambda: gen_body_rot_edge(ref, torch),
    }
    only = set(sys.argv[1:])
    for name, fn in jobs.items():
        if only and name not in only:
            continue
        d = fn()
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **d)
        print(f"wrote {name}.npz")
    meta = {"torch": torch.__version__, "mkl": "2024.2", "generator": "tools/make_golden.py",
            "reference": "shuoshuof/Humanoid-Real-Time-Retarget @ 2024-12-20 (read-only /root/reference)"}
    import scipy
    meta["scipy"] = scipy.__version__
    with open(os.path.join(OUT, "META.json"), "w") as f:
        json.dump(meta, f, indent=2)


if __name__ == "__main__":
    main()
