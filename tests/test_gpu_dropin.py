"""The reference's Python API (retarget.retarget_solver, robot_kinematics_model,
poselib ...skeleton3d / ...rotation3d, retarget.spatial_transform.transform3d)
served by the drop-in modules, called exactly the way the reference's entry
points call it (sim_full_body_teleop.py:115-119, sim_teleop.py:102,
base_retargeter.py:22-58), with CPU tensors in and CPU tensors out."""
import numpy as np
import pytest
import torch

from conftest import frame_stats, golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def poses(gpu):
    from robot_kinematics_model import RobotZeroPose
    return {n: RobotZeroPose.from_asset(n) for n in ("hu_v5", "vtrdyn_full", "vtrdyn")}


def test_zero_pose_global_translation_bit_exact(poses):
    zp = golden("zero_pose")
    for n in ("hu_v5", "vtrdyn_full", "vtrdyn"):
        gt = poses[n].global_translation
        assert gt.device.type == "cpu"
        np.testing.assert_array_equal(gt.numpy(), zp[f"{n}_global_t"])


def test_full_body_pos_per_frame_api(poses):
    import oracle as orc
    from retarget.retarget_solver import VtrdynFullBodyPosRetargeter
    d = golden("full_body_pos_precise")
    zp = golden("zero_pose")
    s = VtrdynFullBodyPosRetargeter(poses["vtrdyn_full"], poses["hu_v5"], precise_gripper=True)
    n = 24
    outs = [s.retarget(torch.from_numpy(d["body"][i]), torch.from_numpy(d["lh"][i]), torch.from_numpy(d["rh"][i]))
            for i in range(n)]
    lr, dof, br = outs[0]
    assert lr.shape == (31, 4) and dof.shape == (30,) and br.shape == (59, 4) and dof.device.type == "cpu"
    dof = np.stack([o[1].numpy() for o in outs])
    odof, olr, obr = orc.full_body_pos(zp["vtrdyn_full_local_t"], zp["vtrdyn_full_global_t"], d["body"][:n],
                                       d["lh"][:n], d["rh"][:n], True)
    np.testing.assert_array_equal(dof, odof)
    np.testing.assert_array_equal(np.stack([o[2].numpy() for o in outs]), obr)
    assert frame_stats(dof, d["dof"][:n])["max"] <= 2e-3
    # accumulated motion + FK of the retargeted motion (base_retargeter.py:22-58)
    assert s.motion_length == n
    np.testing.assert_array_equal(s.motion_dof_pos.numpy(), odof)
    from rtg import assets
    gr, gp = orc.fk(assets.parents("hu_v5"), poses["hu_v5"].local_translation.numpy(), olr, np.zeros((n, 3), np.float32))
    np.testing.assert_array_equal(s.motion_global_rotation.numpy(), gr)
    np.testing.assert_array_equal(s.motion_global_translation.numpy(), gp)


def test_batched_equals_per_frame(poses):
    from retarget.retarget_solver import VtrdynFullBodyPosRetargeter
    d = golden("full_body_pos_binary")
    s = VtrdynFullBodyPosRetargeter(poses["vtrdyn_full"], poses["hu_v5"], precise_gripper=False)
    lr_b, dof_b, br_b = s.retarget_batch(torch.from_numpy(d["body"]).cuda(), torch.from_numpy(d["lh"]).cuda(),
                                         torch.from_numpy(d["rh"]).cuda(), want_body_rot=True)
    assert dof_b.is_cuda and dof_b.shape == (len(d["body"]), 30)
    for i in (0, 7, 63):
        lr, dof, br = s.retarget(torch.from_numpy(d["body"][i]), torch.from_numpy(d["lh"][i]),
                                 torch.from_numpy(d["rh"][i]))
        assert torch.equal(dof, dof_b[i].cpu()) and torch.equal(lr, lr_b[i].cpu()) and torch.equal(br, br_b[i].cpu())


def test_other_solver_classes(poses):
    import oracle as orc
    from rtg import assets
    from retarget.retarget_solver import (HuUpperBodyFromMocapRetarget, Mocap2HuBodyRetargeter,
                                          VtrdynFullBodyRetargeter)
    zp = golden("zero_pose")
    d = golden("upper_body")
    s = HuUpperBodyFromMocapRetarget(poses["vtrdyn"], poses["hu_v5"])
    lr, dof = s.retarget_from_global_translation(torch.from_numpy(d["x"][3]))
    np.testing.assert_array_equal(dof.numpy(), orc.upper_body(zp["vtrdyn_local_t"], d["x"][3:4])[0][0])
    d = golden("full_body_rot")
    s = VtrdynFullBodyRetargeter(poses["vtrdyn_full"], poses["hu_v5"])
    lr, dof = s.retarget(torch.from_numpy(d["body_rot"][5]), torch.from_numpy(d["body_pos"][5]), None,
                         torch.from_numpy(d["lh"][5]), None, torch.from_numpy(d["rh"][5]))
    np.testing.assert_array_equal(dof.numpy(), orc.full_body_rot(zp["vtrdyn_full_local_t"], d["body_rot"][5:6],
                                                                 d["body_pos"][5:6], d["lh"][5:6], d["rh"][5:6])[0][0])
    d = golden("body_rot")
    s = Mocap2HuBodyRetargeter(poses["vtrdyn"], poses["hu_v5"])
    lr, dof = s.retarget_from_pose(torch.from_numpy(d["global_rot"][9]))
    np.testing.assert_array_equal(dof.numpy(), orc.body_rot(assets.parents("vtrdyn"), d["global_rot"][9:10])[0][0])
    assert frame_stats(dof.numpy()[None], d["dof"][9:10])["max"] <= 1e-6


def test_rotation3d_mirror_bit_exact_cpu_in_cpu_out(gpu):
    from poselib.poselib.core import rotation3d as r3
    p = golden("primitives")
    a, b = torch.from_numpy(p["qm_a"]), torch.from_numpy(p["qm_b"])
    out = r3.quat_mul(a, b)
    assert out.device.type == "cpu"
    np.testing.assert_array_equal(out.numpy(), p["quat_mul"])
    np.testing.assert_array_equal(r3.quat_mul_norm(a, b).numpy(), p["quat_mul_norm"])
    np.testing.assert_array_equal(r3.quat_normalize(a).numpy(), p["quat_normalize"])
    np.testing.assert_array_equal(r3.quat_rotate(b, torch.from_numpy(p["qr_v"])).numpy(), p["quat_rotate"])
    q = r3.quat_mul_three(a, b, a)
    np.testing.assert_array_equal(q.numpy(), r3.quat_mul(r3.quat_mul(a, b), a).numpy())
    t = r3.transform_mul(torch.cat([b, torch.ones(len(b), 3)], -1), torch.cat([a, torch.zeros(len(a), 3)], -1))
    assert t.shape == (len(a), 7)


def test_transform3d_mirror(gpu):
    from retarget.spatial_transform import transform3d as tf
    from retarget.robot_config.Hu_v5 import Hu_DOF_AXIS
    p = golden("primitives")
    eye = torch.eye(3)
    v1 = torch.from_numpy(p["rbv_v1"])
    np.testing.assert_array_equal(tf.proj_in_plane(v1[0], eye[1]).numpy(), p["proj_in_plane_y"][0])
    r = tf.radians_between_vecs(v1[2], torch.from_numpy(p["rbv_v2"][2]), torch.from_numpy(p["rbv_n"][2]))
    assert r.dim() == 0 and abs(float(r) - float(p["radians_between_vecs"][2])) <= 2.5e-7
    dof = tf.quat_to_dof_pos(torch.from_numpy(p["dof_q31"][3, 1:]), Hu_DOF_AXIS)
    assert frame_stats(dof.numpy()[None], p["quat_to_dof_pos"][3:4])["max"] <= 2.5e-7
    q1, q2, q3 = tf.quat_in_xyz_axis(torch.from_numpy(p["qxyz_q"][:4]), "XYZ")
    np.testing.assert_array_equal(torch.stack([q1, q2, q3], 1).numpy(), p["quat_in_xyz_axis_XYZ"][:4])
    Z, M = torch.from_numpy(p["cjq5_Z"][:1]), torch.from_numpy(p["cjq5_M"][:1])
    assert tf.cal_joint_quat(Z, M).shape == (1, 4)
    x = torch.arange(6, dtype=torch.float32).reshape(2, 3)
    np.testing.assert_array_equal(tf.coord_transform(x, dir=torch.Tensor([-1, -1, 1])).numpy(),
                                  (x * torch.Tensor([-1, -1, 1])).numpy())


def test_skeleton_state_and_kinematics_mirror(gpu):
    from poselib.poselib.skeleton.skeleton3d import SkeletonState, SkeletonTree
    from robot_kinematics_model import cal_forward_kinematics, cal_local_rotation
    from rtg import assets
    k = golden("kinematics")
    for name in ("hu_v5", "vtrdyn_full"):
        tree = SkeletonTree([str(s) for s in assets.load(name)["node_names"]], torch.from_numpy(assets.parents(name)),
                            torch.from_numpy(assets.local_translation(name)), torch.from_numpy(assets.tree_quat(name)))
        st = SkeletonState.from_rotation_and_root_translation(tree, torch.from_numpy(k[f"{name}_local_rot"]),
                                                              torch.from_numpy(k[f"{name}_root_t"]), is_local=True)
        np.testing.assert_array_equal(st.global_rotation.numpy(), k[f"{name}_state_g_rot"])
        np.testing.assert_array_equal(st.global_translation.numpy(), k[f"{name}_state_g_pos"])
        sg = SkeletonState.from_rotation_and_root_translation(tree, st.global_rotation, st.root_translation,
                                                              is_local=False)
        np.testing.assert_array_equal(sg.local_rotation.numpy(), k[f"{name}_state_local_rot"])
        gr, gp = cal_forward_kinematics(torch.from_numpy(k[f"{name}_local_rot"]), torch.from_numpy(k[f"{name}_root_t"]),
                                        tree.parent_indices, tree.local_translation)
        np.testing.assert_array_equal(gr.numpy(), k[f"{name}_g_rot"])
        np.testing.assert_array_equal(gp.numpy(), k[f"{name}_g_pos"])
        np.testing.assert_array_equal(cal_local_rotation(gr, tree.parent_indices).numpy(), k[f"{name}_inv_local"])


def test_skeleton_state_pickle_roundtrip(gpu):
    import pickle
    from robot_kinematics_model import RobotZeroPose
    from poselib.poselib.skeleton.skeleton3d import SkeletonState
    st = SkeletonState.zero_pose(RobotZeroPose.from_asset("hu_v5").skeleton_tree)
    st2 = pickle.loads(pickle.dumps(st))
    assert torch.equal(st2.global_translation, st.global_translation)


def test_skeleton_motion_from_state(gpu):
    from poselib.poselib.skeleton.skeleton3d import SkeletonMotion, SkeletonState
    from robot_kinematics_model import RobotZeroPose
    m = golden("motion")
    tree = RobotZeroPose.from_asset("hu_v5").skeleton_tree
    st = SkeletonState.from_rotation_and_root_translation(tree, torch.from_numpy(m["local_rot"]),
                                                          torch.from_numpy(m["root_t"]), is_local=True)
    mo = SkeletonMotion.from_skeleton_state(st, fps=30)
    assert mo.tensor.device.type == "cpu" and mo.fps == 30
    np.testing.assert_array_equal(mo.global_velocity.numpy(), m["global_velocity"])
    assert frame_stats(mo.global_angular_velocity.numpy(), m["global_angular_velocity"])["max"] <= 1e-6
    np.testing.assert_array_equal(mo.tensor.numpy()[:, :31 * 4 + 3], m["tensor"][:, :31 * 4 + 3])


def test_hu_forward_model_dropin(gpu):
    """robot_kinematics_model.hu_forward_model.HuForwardModel: reference shapes and clip semantics."""
    import torch
    import oracle as orc
    from robot_kinematics_model.hu_forward_model import HuForwardModel
    from rtg import assets
    from retarget.robot_config import Hu
    d = golden("dof_fk")
    from robot_kinematics_model import RobotZeroPose
    m = HuForwardModel(RobotZeroPose.from_asset("hu").skeleton_tree)
    L = 128
    ang = torch.from_numpy(d["hu_clip_dof"]).reshape(L, 32, 1).cuda()
    rr = torch.from_numpy(d["hu_clip_root_rot"]).reshape(L, 1, 4).cuda()
    rt = torch.from_numpy(d["hu_clip_root_t"]).cuda()
    gr, gp = m.forward_kinematics(motion_joint_angles=ang, motion_root_translation=rt, motion_root_rotation=rr,
                                  clip_angles=True)
    assert gr.shape == (L, 33, 4) and gp.shape == (L, 33, 3) and gr.device.type == "cuda"
    ogr, ogp = orc.dof_fk(assets.parents("hu"), assets.local_translation("hu"), Hu.Hu_DOF_AXIS, d["hu_clip_dof"],
                          d["hu_clip_root_rot"], d["hu_clip_root_t"], Hu.Hu_DOF_LOWER.numpy(), Hu.Hu_DOF_UPPER.numpy())
    np.testing.assert_array_equal(gr.cpu().numpy(), ogr)
    np.testing.assert_array_equal(gp.cpu().numpy(), ogp)
    c = m._clip_angles(ang)
    assert c.shape == ang.shape and bool((c.cpu() <= Hu.Hu_DOF_UPPER.reshape(1, -1, 1) + 1e-6).all())
    m5 = HuForwardModel(RobotZeroPose.from_asset("hu_v5").skeleton_tree)
    with pytest.raises(ValueError):
        m5.forward_kinematics(torch.zeros(2, 30, 1), torch.zeros(2, 3), torch.zeros(2, 1, 4), clip_angles=True)


def test_main_motion_prep_dropin(gpu):
    """retarget.main (legacy motion path): rescale + rebuild through the drop-in classes."""
    import oracle as orc
    from retarget.main import Retarget, RetargetHuV5fromMocap
    from robot_kinematics_model import RobotZeroPose
    from rtg import assets
    d = golden("motion_prep")
    zp = RobotZeroPose.from_asset("vtrdyn")
    m = torch.from_numpy(d["raw"]) * torch.tensor([-1.0, -1.0, 1.0])
    r = Retarget.rescale_motion_to_standard_size(m, zp)
    assert r.device.type == "cpu"
    np.testing.assert_array_equal(r.numpy(), d["rescaled"])
    motion = RetargetHuV5fromMocap(zp, zp)._rebuild_with_vtrdyn_zero_pose(r)
    ogr, ort = orc.rebuild_vtrdyn(assets.parents("vtrdyn"), golden("zero_pose")["vtrdyn_local_t"], d["rescaled"])
    np.testing.assert_array_equal(motion.global_rotation.cpu().numpy(), ogr)
    np.testing.assert_array_equal(motion.root_translation.cpu().numpy(), ort)
    assert motion.global_velocity.shape == (len(ogr), 21, 3)


def test_per_frame_graph_matches_batched(gpu):
    """The teleop per-frame call (host tensors -> captured HIP graph, rtg.realtime.FrameGraph) returns exactly
    the batched solve's rows, frame after frame."""
    from retarget.retarget_solver import VtrdynFullBodyPosRetargeter
    from robot_kinematics_model import RobotZeroPose
    g = golden("full_body_pos_precise")
    hu = VtrdynFullBodyPosRetargeter(RobotZeroPose.from_asset("vtrdyn_full"), RobotZeroPose.from_asset("hu_v5"),
                                     precise_gripper=True, frame_server=False)
    n = 40
    lr_b, dof_b, br_b = hu.retarget_batch(torch.from_numpy(g["body"][:n]), torch.from_numpy(g["lh"][:n]),
                                          torch.from_numpy(g["rh"][:n]), want_body_rot=True)
    for i in range(n):
        lr, dof, br = hu.retarget(torch.from_numpy(g["body"][i]), torch.from_numpy(g["lh"][i]),
                                  torch.from_numpy(g["rh"][i]))
        assert lr.device.type == "cpu" and dof.shape == (30,) and br.shape == (59, 4)
        np.testing.assert_array_equal(dof.numpy(), dof_b[i].numpy())
        np.testing.assert_array_equal(lr.numpy(), lr_b[i].numpy())
        np.testing.assert_array_equal(br.numpy(), br_b[i].numpy())
    assert hu.motion_length == n


def test_frame_server_matches_batched(gpu):
    """The resident per-frame server (rtg_frame_server_launch, rtg.realtime.FrameServer) serves frame after frame
    with exactly the batched solve's rows, relaunches itself after an idle exit, and ends on close() -- with its inbox
    in device memory (rtg_server_inbox_alloc) and in pinned host memory."""
    import time

    from retarget.retarget_solver import VtrdynFullBodyPosRetargeter
    from robot_kinematics_model import RobotZeroPose
    from rtg.realtime import FrameServer
    g = golden("full_body_pos_precise")
    hu = VtrdynFullBodyPosRetargeter(RobotZeroPose.from_asset("vtrdyn_full"), RobotZeroPose.from_asset("hu_v5"),
                                     precise_gripper=True)
    n = 48
    lr_b, dof_b, br_b = hu.retarget_batch(torch.from_numpy(g["body"][:n]), torch.from_numpy(g["lh"][:n]),
                                          torch.from_numpy(g["rh"][:n]), want_body_rot=True)
    large_bar = _large_bar()
    for device_inbox in (True, False):   # the inbox in device memory through the BAR (MI355X), or pinned
        with FrameServer(hu.solver, want_body_rot=True, idle_ms=20, device_inbox=device_inbox) as fs:
            # without a large BAR the library refuses a device inbox and the server keeps a pinned one
            assert (fs._inbox is not None) == (device_inbox and large_bar)
            for i in range(n):
                if i == n // 2:
                    time.sleep(0.1)   # past idle_ms: the server has ended; the next call relaunches it
                    assert fs._ctl[2] == 1
                lr, dof, br = fs(g["body"][i], g["lh"][i], g["rh"][i])
                np.testing.assert_array_equal(dof.numpy(), dof_b[i].numpy())
                np.testing.assert_array_equal(lr.numpy(), lr_b[i].numpy())
                np.testing.assert_array_equal(br.numpy(), br_b[i].numpy())
        assert not fs._running and fs._ctl[2] == 1
    with pytest.raises(ValueError):
        FrameServer(hu.solver, want_body_rot=True)(g["body"][0], g["lh"][0])


def _large_bar() -> bool:
    """Whether the library can hand out a device inbox here (rtg_server_inbox_alloc refuses without a large BAR)."""
    import ctypes

    from rtg._lib import lib
    p = ctypes.c_void_p()
    if lib().rtg_server_inbox_alloc(ctypes.byref(p)) != 0 or not p.value:
        return False
    from rtg import realtime
    realtime._inbox_give(p.value)   # into the process pool (no hipFree: a device-wide synchronize)
    return True


def test_dropping_a_server_while_another_is_resident_returns_at_once(gpu):
    """a FrameServer's release must not synchronize the device.  With a second server resident (its
    stream busy until it idles out, 2 s here), dropping the first one returns in well under that, its device inbox
    goes back to the process pool and the next server takes it, reset to sequence word 0 and serving exactly."""
    import gc
    import time

    from retarget.retarget_solver import VtrdynFullBodyPosRetargeter
    from robot_kinematics_model import RobotZeroPose
    from rtg import realtime
    from rtg.realtime import FrameServer
    g = golden("full_body_pos_precise")
    hu = VtrdynFullBodyPosRetargeter(RobotZeroPose.from_asset("vtrdyn_full"), RobotZeroPose.from_asset("hu_v5"),
                                     precise_gripper=True)
    _, dof_b, _ = hu.retarget_batch(torch.from_numpy(g["body"][:4]), torch.from_numpy(g["lh"][:4]),
                                    torch.from_numpy(g["rh"][:4]))
    resident = FrameServer(hu.solver, idle_ms=2000)
    resident(g["body"][0], g["lh"][0], g["rh"][0])          # launched, and stays resident for 2 s
    a = FrameServer(hu.solver, idle_ms=2000)
    a(g["body"][1], g["lh"][1], g["rh"][1])
    inbox = a._inbox
    a.close()                                              # a's own stream only
    t0 = time.perf_counter()
    del a
    gc.collect()
    dt = time.perf_counter() - t0
    assert dt < 0.5, dt                                    # a device-wide sync would wait ~2 s for `resident`
    if inbox:
        assert inbox in realtime._INBOX_POOL
        b = FrameServer(hu.solver, idle_ms=50)
        assert b._inbox == inbox                           # reused, its sequence word reset to 0
        for i in range(4):
            _, dof, _ = b(g["body"][i], g["lh"][i], g["rh"][i])
            np.testing.assert_array_equal(dof.numpy(), dof_b[i].numpy())
        b.close()
    _, dof, _ = resident(g["body"][2], g["lh"][2], g["rh"][2])
    np.testing.assert_array_equal(dof.numpy(), dof_b[2].numpy())
    resident.close()


def test_per_frame_calls_do_not_stall_device_synchronize(gpu):
    """a torch.cuda.synchronize() between teleop frames returns at once with the one-launch path
    (frame_server=False, nothing resident) and within the server's idle_ms with the resident server -- the default,
    100 ms since round 5 (teleop loops leave 5-33 ms between frames: profiles/r05/teleop/); close() ends it at
    once; one runner serves both retarget() (body_rot) and a caller that drops it."""
    import time

    from retarget.retarget_solver import VtrdynFullBodyPosRetargeter
    from robot_kinematics_model import RobotZeroPose
    g = golden("full_body_pos_precise")
    zf, zh = RobotZeroPose.from_asset("vtrdyn_full"), RobotZeroPose.from_asset("hu_v5")
    for server, idle_ms, bound_s in ((False, 200, 0.05), (True, 10, 0.15), (None, None, 0.25)):
        kw = {} if server is None else dict(frame_server=server, idle_ms=idle_ms)   # None: the defaults
        hu = VtrdynFullBodyPosRetargeter(zf, zh, precise_gripper=True, **kw)
        worst = 0.0
        for i in range(6):
            _, dof, br = hu.retarget(g["body"][i], g["lh"][i], g["rh"][i])
            assert br.shape == (59, 4)
            t0 = time.perf_counter()
            torch.cuda.synchronize()
            worst = max(worst, time.perf_counter() - t0)
        assert worst < bound_s, (server, worst)
        hu.close()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        assert time.perf_counter() - t0 < 0.05
        assert hu._frame_runner is None


def test_main_retarget_from_global_translation(gpu):
    """retarget/main.py RetargetHuV5fromMocap.retarget_from_global_translation (:169-279), unchanged call, against
    the reference run end to end (tests/golden/main_retarget.npz, plot_skeleton_H captured) and against the oracle
    composition of the same chain: coord_transform + rescale -> rebuild -> SkeletonState FK of the rebuilt motion
    -> the arm maps on its rotation 10 and translations (quat_mul_three parent) -> SkeletonState(is_local=True)."""
    import oracle as orc
    import retarget.main as M
    from robot_kinematics_model import RobotZeroPose
    from rtg import assets, ops
    g = golden("main_retarget")
    zv, hu = RobotZeroPose.from_asset("vtrdyn"), RobotZeroPose.from_asset("hu_v5")
    got = []
    hook = M.plot_skeleton_H
    M.plot_skeleton_H = lambda motions, *a, **k: got.extend(motions)
    try:
        r = M.RetargetHuV5fromMocap(zv, hu).retarget_from_global_translation(torch.from_numpy(g["x"]))
    finally:
        M.plot_skeleton_H = hook
    assert r is None and len(got) == 2
    mocap, robot = got
    # oracle composition
    par, zl = assets.parents("vtrdyn"), golden("zero_pose")["vtrdyn_local_t"]
    tq = assets.tree_quat("vtrdyn")
    x = orc.rescale_motion(par, zl, g["x"], dir=[-1.0, -1.0, 1.0])
    gr, rt = orc.rebuild_vtrdyn(par, zl, x)
    _, gp = orc.state_fk(par, tq, zl, orc.state_local_rotation(par, tq, gr), rt)
    np.testing.assert_array_equal(mocap.global_rotation.numpy(), gr)
    np.testing.assert_array_equal(mocap.global_translation.numpy(), gp)
    L = len(gr)
    lr = np.tile(np.float32([0, 0, 0, 1]), (L, 31, 1))
    for links, (sh, el, wr) in (((12, 13, 14, 15), (18, 19, 20)), ((21, 22, 23, 24), (14, 15, 16))):
        pr = orc.shoulder_pr(gp[:, el] - gp[:, sh], np.tile(zl[el], (L, 1)), gr[:, 10])
        parent = orc.quat_mul(orc.quat_mul(gr[:, 10], pr[:, 0]), pr[:, 1])
        ye = orc.elbow_py(gp[:, wr] - gp[:, el], np.tile(zl[wr], (L, 1)), parent)
        for link, q in zip(links, (pr[:, 0], pr[:, 1], ye[:, 0], ye[:, 1])):
            lr[:, link] = q
    lr = orc.quat_normalize(lr.reshape(-1, 4)).reshape(L, 31, 4)
    np.testing.assert_array_equal(robot.local_rotation.numpy(), lr)
    hpar, htq, hzl = assets.parents("hu_v5"), assets.tree_quat("hu_v5"), assets.local_translation("hu_v5")
    ogr, ogp = orc.state_fk(hpar, htq, hzl, lr, np.zeros((L, 3), np.float32))
    np.testing.assert_array_equal(robot.global_rotation.numpy(), ogr)
    np.testing.assert_array_equal(robot.global_translation.numpy(), ogp)
    w, _ = ops.gaussian_taps()
    np.testing.assert_array_equal(robot.global_velocity.numpy(), orc.linear_velocity(ogp, 1 / 30, w))
    # against the reference itself: the mocap side is bit-exact but for VML sqrt's ulp in the Kabsch rows; the
    # arm angles carry VML's acos/sin/cos ulps
    assert frame_stats(mocap.global_rotation.numpy(), g["mocap_g_rot"])["max"] <= 6e-8
    s = frame_stats(robot.local_rotation.numpy(), g["robot_local_rot"])
    assert s["max"] <= 2e-5 and s["exact_elems"] >= 0.9, s
    assert frame_stats(robot.global_translation.numpy(), g["robot_g_pos"])["max"] <= 2e-5


def test_rotation3d_transform3d_full_surface_vs_oracle_and_reference(gpu):
    """Everything rotation3d / transform3d export beyond the solver path, through the drop-in functions (rtg_quat_op_f32
    ops 18-31, rtg_quat_as_euler_f64, rtg_quat_between_f32): bit-exact vs the oracle, and vs the reference's own
    outputs (tests/golden/overlay_extras.npz) exact where no transcendental is involved, within VML's ulps where
    one is.  CPU tensors in, CPU tensors out, like the reference."""
    import oracle as orc
    import poselib.poselib.core.rotation3d as r3
    import retarget.spatial_transform.transform3d as t3
    g = golden("overlay_extras")
    T = torch.from_numpy

    def both(got, o, ref, exact_ref):
        got = got.numpy() if isinstance(got, torch.Tensor) else np.asarray(got)
        np.testing.assert_array_equal(got, o)
        if exact_ref:
            np.testing.assert_array_equal(got, ref)
        else:
            e = np.abs(got.astype(np.float64) - ref)
            assert np.nanmax(e) <= 2.5e-7, np.nanmax(e)

    a, ax = r3.exp_map_to_angle_axis(T(g["em_e"]))
    assert a.device.type == "cpu"
    both(torch.cat([a[:, None], ax], 1), orc.exp_map_to_angle_axis(g["em_e"]), g["exp_map_to_angle_axis"], False)
    both(r3.exp_map_to_quat(T(g["em_e"])), orc.exp_map_to_quat(g["em_e"]), g["exp_map_to_quat"], False)
    both(t3.exp_map_to_quat(T(g["em_e"])), orc.exp_map_to_quat(g["em_e"]), g["t3_exp_map_to_quat"], False)
    both(t3.quat_slerp(T(g["sl_q0"]), T(g["sl_q1"]), T(g["sl_t"])), orc.quat_slerp(g["sl_q0"], g["sl_q1"], g["sl_t"]),
         g["quat_slerp"], False)
    qb = np.concatenate([t3.quat_between_two_vecs(T(g["qb_v1"][i:i + 16]), T(g["qb_v2"][i:i + 16])).numpy()
                         for i in range(0, len(g["qb_v1"]), 16)])   # batch-level identity branch: same chunks
    np.testing.assert_array_equal(qb, g["quat_between_two_vecs"])
    both(torch.stack([r3.quat_from_xyz(T(x.copy())) for x in g["qx_xyz"]]), orc.quat_from_xyz(g["qx_xyz"]),
         g["quat_from_xyz"], True)
    with pytest.raises(AssertionError):
        r3.quat_from_xyz(torch.tensor([1.0, 1.0, 1.0]))                        # rotation3d.py:107
    both(r3.rot_matrix_from_quaternion(T(g["pq_q"])), orc.rot_matrix_from_quaternion(g["pq_q"]),
         g["rot_matrix_from_quaternion"], True)
    both(r3.rot_matrix_det(T(g["det_m"])), orc.rot_matrix_det(g["det_m"]), g["rot_matrix_det"], True)
    for k in ("x", "y", "z", "xy", "xz"):
        both(getattr(r3, f"project_quat_to_axis_{k}")(T(g["pq_q"])), orc.project_quat_to_axis(g["pq_q"], k),
             g[f"project_quat_to_axis_{k}"], False)
    for axis in range(3):
        both(r3.extract_rotation_along_axis(T(g["pq_q"]), axis), orc.extract_rotation_along_axis(g["pq_q"], axis),
             g[f"extract_rotation_along_axis_{axis}"], True)
    for z_up in (True, False):
        np.testing.assert_array_equal(r3.quat_yaw_rotation(T(g["pq_q"]), z_up).numpy(), g[f"quat_yaw_rotation_{int(z_up)}"])
    eu = r3.quat_to_eular(T(g["pq_q"][:256]))
    assert eu.dtype == np.float64
    # float64 out: the device's f64 atan2 / hypot (OCML) are within a few ulp of glibc's, which scipy and the
    # oracle use -- exact agreement is not claimed here (the solver path rounds these angles to f32 first)
    np.testing.assert_allclose(eu, g["quat_to_eular"], rtol=1e-13, atol=1e-12)
    np.testing.assert_allclose(eu, orc.quat_to_eular(g["pq_q"][:256]), rtol=1e-13, atol=1e-12)
    et = r3.euclidean_to_transform(T(g["eu_m"])).numpy()
    o = np.concatenate([orc.quat_from_rotation_matrix(g["eu_m"][:, :3, :3]), g["eu_m"][:, :3, 3]], 1)
    both(et, o, g["euclidean_to_transform"], False)   # quat_from_rotation_matrix's sqrt: VML's ulp
    with pytest.raises(RuntimeError):
        r3.euclidean_inverse(T(g["eu_m"]))                                     # broken in the reference too
