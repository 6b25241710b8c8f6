"""GPU parity: librtg_hip.so vs the oracle (bit-level) and vs the reference's
golden vectors (the reference-noise-bounded statistics of test_oracle_golden.py).

All calls go through the C ABI (rtg._lib via rtg.runtime / rtg.ops)."""
import os

import numpy as np
import pytest
import torch

from conftest import frame_stats, golden

pytestmark = pytest.mark.gpu

TOPOS = ["hu_v5", "vtrdyn", "vtrdyn_full", "noitom"]


def _topo(name):
    from rtg import assets
    from rtg.runtime import Topology
    return Topology(assets.parents(name), assets.local_translation(name), assets.tree_quat(name))


def _np(t):
    return t.detach().cpu().numpy()


# ----------------------------------------------------------------- kinematics
@pytest.mark.parametrize("name", TOPOS)
def test_fk_bit_exact_vs_reference(gpu, name):
    from rtg import ops
    k = golden("kinematics")
    T = _topo(name)
    gr, gp = ops.forward_kinematics(T, k[f"{name}_local_rot"], k[f"{name}_root_t"])
    np.testing.assert_array_equal(_np(gr), k[f"{name}_g_rot"])
    np.testing.assert_array_equal(_np(gp), k[f"{name}_g_pos"])
    loc = ops.local_rotation(T, k[f"{name}_g_rot"])
    np.testing.assert_array_equal(_np(loc), k[f"{name}_inv_local"])


@pytest.mark.parametrize("name", TOPOS)
def test_state_fk_bit_exact_vs_reference(gpu, name):
    from rtg import ops
    k = golden("kinematics")
    T = _topo(name)
    lr = ops.quat_normalize(k[f"{name}_local_rot"])     # SkeletonState stores normalised rotations
    gr, gp = ops.forward_kinematics(T, lr, k[f"{name}_root_t"], state=True)
    np.testing.assert_array_equal(_np(gr), k[f"{name}_state_g_rot"])
    np.testing.assert_array_equal(_np(gp), k[f"{name}_state_g_pos"])
    g = ops.quat_normalize(k[f"{name}_state_g_rot"])
    np.testing.assert_array_equal(_np(ops.local_rotation(T, g, state=True)), k[f"{name}_state_local_rot"])


def test_fk_multi_one_launch_bit_exact(gpu):
    from rtg import ops
    k = golden("kinematics")
    segs = [(_topo(n), k[f"{n}_local_rot"], k[f"{n}_root_t"]) for n in TOPOS]
    outs = ops.forward_kinematics_multi(segs)
    for n, (gr, gp) in zip(TOPOS, outs):
        np.testing.assert_array_equal(_np(gr), k[f"{n}_g_rot"])
        np.testing.assert_array_equal(_np(gp), k[f"{n}_g_pos"])


def test_kinematics_multi_fk_and_inverse_one_launch(gpu):
    """BASELINE config 5 as one launch: FK of the four robot_config skeletons plus inverse FK of the four
    (rtg_kinematics_multi_f32), and inverse FK alone (rtg_local_rotation_multi_f32): bit-exact vs the reference's
    goldens, ragged batch sizes, every segment independent."""
    import oracle as orc
    from rtg import assets, ops, synth
    k = golden("kinematics")
    fk = [(_topo(n), k[f"{n}_local_rot"], k[f"{n}_root_t"]) for n in TOPOS]
    inv = [(_topo(n), k[f"{n}_g_rot"]) for n in TOPOS]
    fouts, iouts = ops.kinematics_multi(fk, inv)
    for n, (gr, gp), loc in zip(TOPOS, fouts, iouts):
        np.testing.assert_array_equal(_np(gr), k[f"{n}_g_rot"])
        np.testing.assert_array_equal(_np(gp), k[f"{n}_g_pos"])
        np.testing.assert_array_equal(_np(loc), k[f"{n}_inv_local"])
    sizes = [1, 63, 65, 1000]
    segs = []
    for n, B in zip(TOPOS, sizes):
        segs.append((_topo(n), synth.random_local_quats(B, len(assets.parents(n)), B)))
    outs = ops.local_rotation_multi(segs)
    for n, (t, g), o in zip(TOPOS, segs, outs):
        np.testing.assert_array_equal(_np(o), orc.local_rotation(assets.parents(n), g))
    with pytest.raises(ValueError):
        ops.kinematics_multi(fk * 2, inv)
    # malformed FK segments raise before any launch (a (J,4) single frame would read B*J*4 floats)
    t_hu = _topo("hu_v5")
    with pytest.raises(ValueError):
        ops.kinematics_multi([(t_hu, k["hu_v5_local_rot"][0], k["hu_v5_root_t"][0])], [])
    with pytest.raises(ValueError):
        ops.kinematics_multi([(t_hu, k["hu_v5_local_rot"], k["hu_v5_root_t"][:2])], [])
    with pytest.raises(ValueError):
        ops.kinematics_multi([], [(t_hu, k["hu_v5_g_rot"][0])])


def test_fk_large_batch_vs_oracle(gpu):
    import oracle as orc
    from rtg import assets, ops, synth
    B = 50000
    lr = synth.random_local_quats(B, 31, 11)
    rt = np.random.default_rng(3).normal(0, 0.3, (B, 3)).astype(np.float32)
    gr, gp = ops.forward_kinematics(_topo("hu_v5"), lr, rt)
    ogr, ogp = orc.fk(assets.parents("hu_v5"), assets.local_translation("hu_v5"), lr, rt)
    np.testing.assert_array_equal(_np(gr), ogr)
    np.testing.assert_array_equal(_np(gp), ogp)


def test_fk_empty_and_single(gpu):
    from rtg import ops
    T = _topo("hu_v5")
    gr, gp = ops.forward_kinematics(T, np.zeros((0, 31, 4), np.float32), np.zeros((0, 3), np.float32))
    assert gr.shape == (0, 31, 4) and gp.shape == (0, 31, 3)
    k = golden("kinematics")
    gr, gp = ops.forward_kinematics(T, k["hu_v5_local_rot"][:1], k["hu_v5_root_t"][:1])
    np.testing.assert_array_equal(_np(gr), k["hu_v5_g_rot"][:1])


def _random_tree(rng, J, kind):
    """Parent arrays that stress the streaming-FK slot schedule: 'bushy' (random
    earlier parents, many live branch points), 'star' (20 chains hanging off the
    root, interleaved -> more live slots than the kernel keeps, lane-walk fallback),
    'chain' (no branch points)."""
    if kind == "chain":
        return np.arange(-1, J - 1, dtype=np.int32)
    if kind == "star":
        par = np.empty(J, np.int32)
        par[0] = -1
        nch = 20
        for j in range(1, J):
            par[j] = 0 if j <= nch else j - nch   # chain c: 0 -> c -> c+20 -> ...
        return par
    par = np.empty(J, np.int32)
    par[0] = -1
    for j in range(1, J):
        par[j] = rng.integers(0, j)
    return par


@pytest.mark.parametrize("kind,J", [("bushy", 31), ("bushy", 97), ("star", 81), ("chain", 17), ("chain", 1),
                                    ("bushy", 36), ("bushy", 37), ("bushy", 64), ("chain", 64), ("star", 60),
                                    ("bushy", 65)])
def test_fk_random_topologies_vs_oracle(gpu, kind, J):
    """Any parent-indexed tree (parents[j] < j): FK, inverse FK and the state
    variants agree bit for bit with the oracle, on ragged batch sizes."""
    import oracle as orc
    from rtg import ops
    from rtg.runtime import Topology
    rng = np.random.default_rng(J * 7 + len(kind))
    par = _random_tree(rng, J, kind)
    lt = rng.normal(0, 0.2, (J, 3)).astype(np.float32)
    tq = ops.quat_normalize(rng.normal(size=(J, 4)).astype(np.float32))
    tq = tq.cpu().numpy() if hasattr(tq, "cpu") else tq
    T = Topology(par, lt, tq)
    for B in (1, 63, 65, 1000):
        lr = np.ascontiguousarray(rng.normal(size=(B, J, 4)).astype(np.float32))
        rt = rng.normal(0, 0.3, (B, 3)).astype(np.float32)
        gr, gp = ops.forward_kinematics(T, lr, rt)
        ogr, ogp = orc.fk(par, lt, lr, rt)
        np.testing.assert_array_equal(_np(gr), ogr)
        np.testing.assert_array_equal(_np(gp), ogp)
        np.testing.assert_array_equal(_np(ops.local_rotation(T, ogr)), orc.local_rotation(par, ogr))
        nlr = _np(ops.quat_normalize(lr))
        sgr, sgp = ops.forward_kinematics(T, nlr, rt, state=True)
        osgr, osgp = orc.state_fk(par, tq, lt, nlr, rt)
        np.testing.assert_array_equal(_np(sgr), osgr)
        np.testing.assert_array_equal(_np(sgp), osgp)
        ng = _np(ops.quat_normalize(osgr))
        np.testing.assert_array_equal(_np(ops.local_rotation(T, ng, state=True)),
                                      orc.state_local_rotation(par, tq, ng))


def test_fk_positions_at_any_alignment(gpu):
    """The lane-group FK stores a tile's positions as dwordx4 pieces when the position rows are 16-byte aligned and
    dword by dword otherwise: a g_pos 4 bytes into its buffer (a (B, J, 3) view at an odd row offset) gives the same
    bits, and the floats around the rows stay untouched."""
    import ctypes

    import oracle as orc
    from rtg import assets, synth
    from rtg._lib import check, lib
    from rtg.runtime import ptr, stream_handle
    T = _topo("hu_v5")
    for B in (16, 1000):
        lr = torch.from_numpy(synth.random_local_quats(B, 31, 12)).cuda()
        rt = torch.from_numpy(np.random.default_rng(4).normal(0, 0.3, (B, 3)).astype(np.float32)).cuda()
        gr = torch.empty((B, 31, 4), device="cuda")
        buf = torch.full((B * 31 * 3 + 2,), 7.0, device="cuda")
        check(lib().rtg_fk_f32(T.handle, ptr(lr), ptr(rt), B, ptr(gr), ctypes.c_void_p(buf.data_ptr() + 4),
                               stream_handle()))
        torch.cuda.synchronize()
        ogr, ogp = orc.fk(assets.parents("hu_v5"), assets.local_translation("hu_v5"), lr.cpu().numpy(), rt.cpu().numpy())
        b = buf.cpu().numpy()
        assert b[0] == 7.0 and b[-1] == 7.0
        np.testing.assert_array_equal(b[1:-1].reshape(B, 31, 3), ogp)
        np.testing.assert_array_equal(_np(gr), ogr)


DOF_FK_CASES = [("hu_clip", "hu"), ("hu_noclip", "hu"), ("hu_v5_noclip", "hu_v5")]


def _dof_model(d, tag, name):
    from rtg.runtime import DofModel
    lo = d[f"{tag}_lower"] if f"{tag}_lower" in d else None
    hi = d[f"{tag}_upper"] if f"{tag}_upper" in d else None
    return DofModel(_topo(name), d[f"{tag}_axis"], lo, hi), lo, hi


@pytest.mark.parametrize("tag,name", DOF_FK_CASES)
def test_dof_fk_vs_oracle_and_reference(gpu, tag, name):
    """HuForwardModel.forward_kinematics (hu_forward_model.py:17-33) in one launch: bit-exact vs the oracle on
    the golden inputs and on 20001 random frames (angles far outside the limits); vs the reference within the
    VML sin/cos residual pinned in test_oracle_golden.py."""
    import oracle as orc
    from rtg import assets, ops
    d = golden("dof_fk")
    model, lo, hi = _dof_model(d, tag, name)
    clip = lo is not None
    par, lt = assets.parents(name), assets.local_translation(name)
    gr, gp = ops.dof_forward_kinematics(model, d[f"{tag}_dof"], d[f"{tag}_root_rot"], d[f"{tag}_root_t"], clip=clip)
    ogr, ogp = orc.dof_fk(par, lt, d[f"{tag}_axis"], d[f"{tag}_dof"], d[f"{tag}_root_rot"], d[f"{tag}_root_t"], lo, hi)
    np.testing.assert_array_equal(_np(gr), ogr)
    np.testing.assert_array_equal(_np(gp), ogp)
    for got, want in ((_np(gr), d[f"{tag}_g_rot"]), (_np(gp), d[f"{tag}_g_pos"])):
        assert np.abs(got - want).max() <= 2e-6
    rng = np.random.default_rng(17)
    B, n = 20001, model.num_dofs
    dof = rng.uniform(-4, 4, (B, n)).astype(np.float32)
    rr = rng.normal(size=(B, 4)).astype(np.float32)
    rt = rng.normal(0, 0.3, (B, 3)).astype(np.float32)
    gr, gp = ops.dof_forward_kinematics(model, dof, rr, rt, clip=clip)
    ogr, ogp = orc.dof_fk(par, lt, d[f"{tag}_axis"], dof, rr, rt, lo, hi)
    np.testing.assert_array_equal(_np(gr), ogr)
    np.testing.assert_array_equal(_np(gp), ogp)


def test_dof_fk_edge_angles(gpu):
    """The joint rotations' fast path (N-way groups, the near-1.0f normalisation table) against the oracle on the
    angles that leave it: +-0, subnormal and tiny angles (subnormal sin products), +-pi and odd multiples (cos near
    0, the sign flip), huge, +-inf and NaN, mixed into random frames so every group has some; clip off and on."""
    import oracle as orc
    from rtg import assets, ops
    from rtg.runtime import DofModel
    from retarget.robot_config import Hu_v5
    T = _topo("hu_v5")
    par, lt = assets.parents("hu_v5"), assets.local_translation("hu_v5")
    n = T.num_joints - 1
    edge = np.array([0.0, -0.0, 1e-45, -1e-45, 1e-38, 3e-39, -2e-30, 1e-7, np.pi, -np.pi, 3 * np.pi, 2 * np.pi,
                     np.float32(np.pi) * np.float32(1 + 2 ** -23), 1e5, -3e7, 1e30, np.inf, -np.inf, np.nan,
                     4.0, -4.0], np.float32)
    rng = np.random.default_rng(23)
    B = 4099
    dof = rng.uniform(-4, 4, (B, n)).astype(np.float32)
    mask = rng.random((B, n)) < 0.15
    dof[mask] = rng.choice(edge, mask.sum())
    dof[:len(edge)] = edge[:, None]   # whole frames of one edge value
    rr = rng.normal(size=(B, 4)).astype(np.float32)
    rt = rng.normal(0, 0.3, (B, 3)).astype(np.float32)
    lo = np.full(n, -2.5, np.float32)
    hi = np.full(n, 2.5, np.float32)
    for lim in (None, (lo, hi)):
        model = DofModel(T, Hu_v5.Hu_DOF_AXIS, *(lim or (None, None)))
        gr, gp = ops.dof_forward_kinematics(model, dof, rr, rt, clip=lim is not None)
        ogr, ogp = orc.dof_fk(par, lt, np.asarray(Hu_v5.Hu_DOF_AXIS), dof, rr, rt, *(lim or (None, None)))
        np.testing.assert_array_equal(_np(gr), ogr)
        np.testing.assert_array_equal(_np(gp), ogp)


def test_dof_fk_roundtrip_with_retargeted_dofs(gpu):
    """Closing the loop: the retargeted Hu v5 DOFs of the golden frames, driven through the
    joint-angle model, reproduce FK of the solver's own local rotations (identity root)."""
    from rtg import _lib, assets, ops
    from rtg.runtime import DofModel, Solver
    from retarget.robot_config import Hu_v5
    zp = golden("zero_pose")
    g = golden("full_body_pos_precise")
    S = Solver(_lib.SOLVER_FULL_BODY_POS, zp["vtrdyn_full_local_t"], zp["vtrdyn_full_global_t"],
               assets.parents("vtrdyn_full"), True)
    dof, lr, _ = S.retarget([torch.from_numpy(g[k]).cuda() for k in ("body", "lh", "rh")], want_local_rot=True)
    T = _topo("hu_v5")
    B = lr.shape[0]
    root_rot = np.tile(np.array([0, 0, 0, 1], np.float32), (B, 1))
    root_t = np.zeros((B, 3), np.float32)
    gr, gp = ops.dof_forward_kinematics(DofModel(T, Hu_v5.Hu_DOF_AXIS), dof, root_rot, root_t)
    lr = _np(lr).copy()
    lr[:, 0] = root_rot
    fr, fp = ops.forward_kinematics(T, lr, root_t)
    # exp-map -> angle -> angle-axis is not an exact inverse in f32 (DOFs 18/19/27/28 are prismatic:
    # the gripper links rotate by their metre value); compare the rotational chain's positions loosely
    assert np.abs(_np(gp) - _np(fp))[:, :18].max() < 1e-4


def test_motion_prep_vs_oracle_and_reference(gpu):
    """retarget/main.py prep: rescale + quat_between_two_vecs + rebuild, bit-exact vs the
    oracle (golden motion and 50000 random frames); rescale / quat_between bit-exact vs the reference."""
    import oracle as orc
    from rtg import assets, ops
    d = golden("motion_prep")
    zl = golden("zero_pose")["vtrdyn_local_t"]
    par = assets.parents("vtrdyn")
    T = _topo("vtrdyn")
    r = _np(ops.rescale_motion(T, d["raw"], dir=[-1.0, -1.0, 1.0]))
    np.testing.assert_array_equal(r, d["rescaled"])
    np.testing.assert_array_equal(_np(ops.quat_between_two_vecs(d["qb_v1"], d["qb_v2"])), d["qb"])
    np.testing.assert_array_equal(_np(ops.quat_between_two_vecs(d["qb_v1"][:4], np.zeros((4, 3), np.float32))),
                                  d["qb_zero"])
    gr, rt = ops.rebuild_vtrdyn(T, d["rescaled"])
    ogr, ort = orc.rebuild_vtrdyn(par, zl, d["rescaled"])
    np.testing.assert_array_equal(_np(gr), ogr)
    np.testing.assert_array_equal(_np(rt), ort)
    rng = np.random.default_rng(5)
    x = (d["raw"][rng.integers(0, len(d["raw"]), 50000)] * rng.uniform(0.7, 1.3, (50000, 1, 1))
         + rng.normal(0, 0.02, (50000, 21, 3))).astype(np.float32)
    x[7, 12] = x[7, 11]                       # a zero-length bone in one frame: NaN quat there, as the reference
    r = _np(ops.rescale_motion(T, x, dir=[-1.0, -1.0, 1.0]))
    orr = orc.rescale_motion(par, zl, x, dir=[-1.0, -1.0, 1.0])
    np.testing.assert_array_equal(r, orr)
    gr, rt = ops.rebuild_vtrdyn(T, orr)
    ogr, ort = orc.rebuild_vtrdyn(par, zl, orr)
    np.testing.assert_array_equal(_np(gr), ogr)
    np.testing.assert_array_equal(_np(rt), ort)
    y = x.copy()
    y[:, 12] = y[:, 11]                       # degenerate for EVERY frame: the batch-level identity branch
    gr, _ = ops.rebuild_vtrdyn(T, y)
    ogr, _ = orc.rebuild_vtrdyn(par, zl, y)
    np.testing.assert_array_equal(_np(gr), ogr)
    assert (ogr[:, 11] == np.array([0, 0, 0, 1], np.float32)).all()


def test_fast_exact_sqrt_and_reciprocal_exhaustive(gpu):
    """csrc/rtg_math.cuh's cr_sqrt (round 5: v_sqrt_f32 + two residual fmas; v_sqrt_f64 + Newton below 2^-96) and
    rcp64/mulr (v_rcp_f64 + Newton, subnormal quotients via IEEE division) against IEEE f32 sqrt / division on the
    device: all 2^32 sqrt inputs, cr_acos (round 5: f64 asin kernel + rounding test) against the libm f64 acos for
    every f32 input, the atan2-free 'XYZ' Euler split (round 5) against the scipy restatement on 2^30 quaternions,
    2^32 random division pairs and all special-value pairs; the exp-map angle table for every f32 w; and
    sqrt_clamp_rcp (one v_rsq_f64, round 3) bitwise equal to clamp(cr_sqrt) + rcp64 for every f32 input; the
    grouped mulr_k (one subnormal branch per group of quotients, round 3) against IEEE division
    (tools/check_fastmath.hip)."""
    import subprocess
    import __graft_entry__ as ge
    exe = ge.FASTMATH_BIN
    if not os.path.exists(exe) or os.path.getmtime(exe) < os.path.getmtime(ge.FASTMATH_SRC):
        ge.build_fastmath_check()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.count(" 0 mismatches") == 8, r.stdout + r.stderr


# ----------------------------------------------------------------- primitives
def test_quaternion_algebra_bit_exact(gpu):
    from rtg import ops
    p = golden("primitives")
    np.testing.assert_array_equal(_np(ops.quat_mul(p["qm_a"], p["qm_b"])), p["quat_mul"])
    np.testing.assert_array_equal(_np(ops.quat_mul_norm(p["qm_a"], p["qm_b"])), p["quat_mul_norm"])
    np.testing.assert_array_equal(_np(ops.quat_normalize(p["qm_a"])), p["quat_normalize"])
    np.testing.assert_array_equal(_np(ops.quat_rotate(p["qm_b"], p["qr_v"])), p["quat_rotate"])


def test_transcendental_primitives_vs_oracle(gpu):
    import oracle as orc
    from rtg import ops
    p = golden("primitives")
    cases = [
        (ops.quat_from_angle_axis(p["qaa_angle"], p["qaa_axis"]), orc.quat_from_angle_axis(p["qaa_angle"], p["qaa_axis"])),
        (ops.quat_from_rotation_matrix(p["qrm_m"]), orc.quat_from_rotation_matrix(p["qrm_m"])),
        (ops.quat_to_dof_pos_hu(p["dof_q31"]), orc.quat_to_dof_pos(p["dof_q31"])),
        (ops.radians_between_vecs(p["rbv_v1"], p["rbv_v2"], p["rbv_n"]), orc.radians_between(p["rbv_v1"], p["rbv_v2"], p["rbv_n"])),
        (torch.stack(ops.cal_shoulder_pr(p["sh_v1"], p["sh_v0"], p["sh_parent"]), -2), orc.shoulder_pr(p["sh_v1"], p["sh_v0"], p["sh_parent"])),
        (torch.stack(ops.cal_elbow_py(p["sh_v1"], p["el_v0"], p["sh_parent"]), -2), orc.elbow_py(p["sh_v1"], p["el_v0"], p["sh_parent"])),
    ]
    for seq in ("XYZ", "YXZ", "ZYX"):
        cases.append((torch.stack(ops.quat_in_xyz_axis(p["qxyz_q"], seq), -2), orc.quat_in_xyz_axis(p["qxyz_q"], seq)))
    for npts in (3, 5):
        cases.append((ops.cal_joint_quat(p[f"cjq{npts}_Z"], p[f"cjq{npts}_M"]), orc.cal_joint_quat(p[f"cjq{npts}_Z"], p[f"cjq{npts}_M"])))
    for i, (g, o) in enumerate(cases):   # bit for bit (NaN == NaN)
        np.testing.assert_array_equal(_np(g), o, err_msg=f"case {i}")


def test_kabsch_sgesdd_random_and_degenerate_vs_oracle(gpu):
    """The device sgesdd restatement (rtg_math.cuh la_gesdd3) against the oracle's (rtg_oracle.c la_gesdd3),
    bit for bit, on 3- and 5-point fits: well-conditioned rotations with noise, coplanar / collinear point sets
    (rank 2 and 1), reflections, tiny (sgesdd's 2^-40 rescale) and huge scales, exact zeros and duplicates."""
    import oracle as orc
    from rtg import ops
    rng = np.random.default_rng(11)
    for npts in (3, 5):
        n = 16384
        Z = rng.standard_normal((n, npts, 3)).astype(np.float32) * 0.1
        ang = rng.uniform(0, np.pi, n)
        ax = rng.standard_normal((n, 3))
        ax /= np.linalg.norm(ax, axis=1, keepdims=True)
        q = np.concatenate([ax * np.sin(ang / 2)[:, None], np.cos(ang / 2)[:, None]], 1).astype(np.float32)
        M = orc.quat_rotate(np.repeat(q, npts, 0), Z.reshape(-1, 3)).reshape(n, npts, 3)
        M = (M + rng.standard_normal(M.shape) * 2e-3).astype(np.float32)
        k = n // 8
        M[0:k, :, 2] = 0.0                                    # coplanar motion points
        M[k:2 * k] = M[k:2 * k, :1] * rng.uniform(0.5, 2, (k, npts, 1)).astype(np.float32)   # collinear
        M[2 * k:3 * k, :, 0] *= -1.0                          # mirrored: det(U Vt) < 0 branch
        M[3 * k:4 * k] *= np.float32(1e-12)                   # below sgesdd's smlnum: rescaled
        M[4 * k:4 * k + 64] = 0.0                             # all-zero fit
        M[4 * k + 64:4 * k + 128, 1] = M[4 * k + 64:4 * k + 128, 0]   # duplicated point
        M[5 * k:6 * k] *= np.float32(1e3)
        g = _np(ops.cal_joint_quat(Z, M))
        o = orc.cal_joint_quat(Z, M)
        bad = ~np.all((g == o) | (np.isnan(g) & np.isnan(o)), axis=1)
        assert not bad.any(), (npts, int(bad.sum()), np.nonzero(bad)[0][:8])


@pytest.mark.parametrize("name,inp", [("quat_to_exp_map", "em_q"), ("quat_to_angle_axis", "em_q"),
                                      ("normalize_angle", "na_x"), ("quat_abs", "qa_q"), ("quat_unit", "qa_q"),
                                      ("quat_angle_axis", "qaa_q")])
def test_expmap_family_vs_oracle_and_reference(gpu, name, inp):
    """RTG_OP 7, 13-17 (rotation3d.py:41-56, 230-240, 582-627) through rtg_quat_op_f32: bit-exact vs the oracle
    on the golden inputs (w < 0, w = +-1, the 1e-5 sin_theta deadzone, w = 0.25 and its neighbours -- the angle
    table's edge), and within VML's ulp of the reference."""
    import oracle as orc
    from rtg import ops
    g = golden("expmap")
    x = g[inp]
    dev = ops.__dict__[name](x)
    if isinstance(dev, tuple):
        dev = torch.cat([dev[0].unsqueeze(-1), dev[1]], -1)
    got = _np(dev).reshape(len(x), -1)
    o = getattr(orc, name)(x).reshape(len(x), -1)
    np.testing.assert_array_equal(got, o)
    s = frame_stats(got, g[name].reshape(got.shape))
    assert s["max"] <= 8e-7, s


def test_proj_in_plane_and_reference(gpu):
    from rtg import ops
    p = golden("primitives")
    e = torch.eye(3)
    np.testing.assert_array_equal(_np(ops.proj_in_plane(p["rbv_v1"], e[1])), p["proj_in_plane_y"])
    np.testing.assert_array_equal(_np(ops.proj_in_plane(p["rbv_v1"], e[2])), p["proj_in_plane_z"])
    with pytest.raises(AssertionError):
        ops.proj_in_plane(p["rbv_v1"], torch.zeros(3))


# ----------------------------------------------------------------- solvers
def _solver(kind, precise=False):
    from rtg import _lib
    from rtg.runtime import Solver
    zp = golden("zero_pose")
    from rtg import assets
    if kind in (_lib.SOLVER_FULL_BODY_POS, _lib.SOLVER_FULL_BODY_ROT):
        return Solver(kind, zp["vtrdyn_full_local_t"], zp["vtrdyn_full_global_t"], assets.parents("vtrdyn_full"), precise)
    return Solver(kind, zp["vtrdyn_local_t"], zp["vtrdyn_global_t"], assets.parents("vtrdyn"), precise)


def _dev(*arrs):
    return [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in arrs]


# reference-vs-port bounds: the oracle's measured residual rounded up in the third digit (test_oracle_golden.py BOUNDS;
# the GPU is bit-identical to the oracle, so it meets exactly these).  What is left is MKL VML's acos / sin / cos /
# sqrt rounding (test_oracle_golden.py::test_vml_attribution; tools/vml_scan.py: no rounding rule reproduces it)
GOLD_BOUNDS = {
    "full_body_pos_precise": dict(max=2.13e-5, p99=5.52e-6, frac=4 / 512),
    "full_body_pos_binary": dict(max=3.58e-5, p99=4.05e-6, frac=1 / 128),
    "upper_body": dict(max=8.64e-5, p99=1.16e-5, frac=7 / 512),
    "full_body_rot": dict(max=3.27e-5, p99=7.63e-6, frac=2 / 256),
    "body_rot": dict(max=1.2e-7, p99=1.2e-7, frac=0.0),
}


def _check_gold(name, dof_gpu, dof_ref):
    s = frame_stats(dof_gpu, dof_ref)
    b = GOLD_BOUNDS[name]
    assert s["max"] <= b["max"] and s["p99_frame"] <= b["p99"] and s["frac_frames_gt_1e5"] <= b["frac"], (name, s)
    return s


@pytest.mark.parametrize("precise", [True, False])
def test_full_body_pos_solver(gpu, precise):
    import oracle as orc
    from rtg import _lib
    name = "full_body_pos_precise" if precise else "full_body_pos_binary"
    d = golden(name)
    zp = golden("zero_pose")
    S = _solver(_lib.SOLVER_FULL_BODY_POS, precise)
    dof, lr, br = S.retarget(_dev(d["body"], d["lh"], d["rh"]), want_local_rot=True, want_body_rot=True)
    odof, olr, obr = orc.full_body_pos(zp["vtrdyn_full_local_t"], zp["vtrdyn_full_global_t"], d["body"], d["lh"],
                                       d["rh"], precise)
    np.testing.assert_array_equal(_np(dof), odof)   # GPU == oracle, bit for bit
    np.testing.assert_array_equal(_np(lr), olr)
    np.testing.assert_array_equal(_np(br), obr)
    _check_gold(name, _np(dof), d["dof"])
    np.testing.assert_array_equal(_np(dof)[:, list(range(11)) + [29]], 0.0)


@pytest.mark.parametrize("name,kind", [("upper_body", 1), ("full_body_rot", 2), ("body_rot", 3)])
def test_other_solvers(gpu, name, kind):
    import oracle as orc
    from rtg import assets
    d = golden(name)
    zp = golden("zero_pose")
    S = _solver(kind)
    if kind == 1:
        dof, lr, _ = S.retarget(_dev(d["x"]), want_local_rot=True)
        odof, olr = orc.upper_body(zp["vtrdyn_local_t"], d["x"])
    elif kind == 2:
        dof, lr, _ = S.retarget(_dev(d["body_rot"], d["body_pos"], d["lh"], d["rh"]), want_local_rot=True)
        odof, olr = orc.full_body_rot(zp["vtrdyn_full_local_t"], d["body_rot"], d["body_pos"], d["lh"], d["rh"])
    else:
        dof, lr, _ = S.retarget(_dev(d["global_rot"]), want_local_rot=True)
        odof, olr = orc.body_rot(assets.parents("vtrdyn"), d["global_rot"])
    np.testing.assert_array_equal(_np(dof), odof)
    np.testing.assert_array_equal(_np(lr), olr)
    _check_gold(name, _np(dof), d["dof"])


@pytest.mark.parametrize("name,kind", [("full_body_pos_precise", 0), ("upper_body", 1), ("full_body_rot", 2),
                                       ("body_rot", 3)])
def test_solver_batch_invariance(gpu, name, kind):
    """A frame's result does not depend on its batch or its position in the 128-frame tile: the golden frames
    tiled to a ragged 131072+77-frame batch give the same bits, DOFs and local rotations, as the golden batch."""
    d = golden(name)
    ins = {0: ("body", "lh", "rh"), 1: ("x",), 2: ("body_rot", "body_pos", "lh", "rh"), 3: ("global_rot",)}[kind]
    S = _solver(kind, True) if kind == 0 else _solver(kind)
    small = _dev(*[d[k] for k in ins])
    n = small[0].shape[0]
    B = 131072 + 77
    idx = torch.arange(B, device="cuda") % n
    big = [t[idx].contiguous() for t in small]
    dof_s, lr_s, _ = S.retarget(small, want_local_rot=True)
    dof_b, lr_b, _ = S.retarget(big, want_local_rot=True)
    assert torch.equal(dof_b, dof_s[idx]) and torch.equal(lr_b, lr_s[idx])


def test_config2_batch4096_vs_oracle(gpu):
    """BASELINE config 2: one 4096-frame batch (device-generated) through the drop-in batched path, every frame
    bit-exact with the oracle."""
    import oracle as orc
    from rtg import _lib, ops
    zp = golden("zero_pose")
    body, lh, rh = ops.synth_full_body(_topo("vtrdyn_full"), 4096, seed=4096)
    S = _solver(_lib.SOLVER_FULL_BODY_POS, True)
    dof, _, _ = S.retarget([body, lh, rh])
    odof, _, _ = orc.full_body_pos(zp["vtrdyn_full_local_t"], zp["vtrdyn_full_global_t"], _np(body), _np(lh),
                                   _np(rh), True, want_rot=False)
    np.testing.assert_array_equal(_np(dof), odof)


@pytest.mark.parametrize("layout", ["aos", "soa"])
def test_quad_tile_ragged_batches_vs_oracle(gpu, layout):
    """k_fbp_quad (2 <= B <= RTG_QUAD_MAX_B: one frame per lane quad; 8 frames per block up to RTG_QUAD8_MAX_B,
    16 above) on ragged batch sizes: DOFs, local and body rotations bit-exact with the oracle, in both input layouts,
    including a NaN frame the reference raises on inside a partial last tile (NaNs compared as NaN; its status code
    bit for bit)."""
    import oracle as orc
    from rtg import _lib, ops
    from rtg.runtime import frame_status
    zp = golden("zero_pose")
    S = _solver(_lib.SOLVER_FULL_BODY_POS, True)

    def bits(a):
        a = np.ascontiguousarray(a, np.float32)
        return np.where(np.isnan(a), np.uint32(0x7FC00000), a.view(np.uint32))

    for B in (2, 15, 16, 17, 47, 4089):
        body, lh, rh = ops.synth_full_body(_topo("vtrdyn_full"), B, seed=B)
        if B in (47, 4089):
            lh[B - 2, 2] = float("nan")   # a frame of the partial last tile: its left wrist fit refuses
        ins = [body, lh, rh] if layout == "aos" else [t.permute(1, 2, 0).contiguous() for t in (body, lh, rh)]
        dof, lr, br = S.retarget(ins, want_local_rot=True, want_body_rot=True, layout=layout)
        odof, olr, obr = orc.full_body_pos(zp["vtrdyn_full_local_t"], zp["vtrdyn_full_global_t"], _np(body),
                                           _np(lh), _np(rh), True)
        np.testing.assert_array_equal(bits(_np(dof)), bits(odof), err_msg=f"B={B}")
        np.testing.assert_array_equal(frame_status(dof).cpu().numpy(), orc.frame_status(odof), err_msg=f"B={B}")
        np.testing.assert_array_equal(bits(_np(lr)), bits(olr), err_msg=f"B={B}")
        np.testing.assert_array_equal(bits(_np(br)), bits(obr), err_msg=f"B={B}")
        assert (orc.frame_status(odof) != 0).sum() == (1 if B in (47, 4089) else 0)


@pytest.mark.parametrize("kind", [0, 1, 2, 3])
def test_soa_layout_matches_aos(gpu, kind):
    """RTG_LAYOUT_SOA inputs ((P, C, B) component planes) give the same bits as the reference's (B, P, C) rows,
    for every solver kind; the synthetic producer emits SoA directly, bit-identical to its AoS output."""
    from rtg import _lib, ops
    T = _topo("vtrdyn_full")
    B = 128 * 37 + 5
    body, lh, rh, rot = ops.synth_full_body(T, B, seed=7, want_rot=True)
    sb, sl, sr, srot = ops.synth_full_body(T, B, seed=7, want_rot=True, layout="soa")
    for a, s in ((body, sb), (lh, sl), (rh, sr), (rot, srot)):
        assert torch.equal(a.permute(1, 2, 0), s)
    ins = {0: ([body, lh, rh], [sb, sl, sr]), 1: ([body], [sb]), 2: ([rot, body, lh, rh], [srot, sb, sl, sr]),
           3: ([rot], [srot])}[kind]
    S = _solver(kind, True) if kind == 0 else _solver(kind)
    d_aos, lr_aos, _ = S.retarget(ins[0], want_local_rot=True)
    d_soa, lr_soa, _ = S.retarget(ins[1], want_local_rot=True, layout="soa")
    assert torch.equal(d_aos, d_soa) and torch.equal(lr_aos, lr_soa)


def test_solver_rejects_bad_out_dof_and_device(gpu):
    """out_dof must be a contiguous float32 (B,30) tensor on the solver's device."""
    from rtg import _lib, ops
    body, lh, rh = ops.synth_full_body(_topo("vtrdyn_full"), 64, seed=1)
    S = _solver(_lib.SOLVER_FULL_BODY_POS, True)
    for bad in (torch.empty(64, 29, device="cuda"), torch.empty(64, 30, device="cuda", dtype=torch.float64),
                torch.empty(30, 64, device="cuda").t(), torch.empty(64, 30)):
        with pytest.raises(ValueError):
            S.retarget([body, lh, rh], out_dof=bad)
    with pytest.raises(ValueError):
        S.retarget([body.cpu(), lh.cpu(), rh.cpu()])


def test_ingest_soa_matches_aos(gpu):
    from rtg import ingest
    rng = np.random.default_rng(3)
    B = 65536 + 37   # ragged last tiles (16-frame AoS, 32-frame SoA)
    b23 = rng.standard_normal((B, 23, 3)).astype(np.float32)
    b23[[5, 64, B - 1]] = 0.0   # frames without data in the first, second and last tiles
    l20, r20 = (rng.standard_normal((B, 20, 3)).astype(np.float32) for _ in range(2))
    a = ingest.reindex_frames(b23, l20, r20)
    s = ingest.reindex_frames(b23, l20, r20, layout="soa")
    for x, y in zip(a[:3], s[:3]):
        assert torch.equal(x.permute(1, 2, 0), y)
    assert torch.equal(a[3], s[3])
    np.testing.assert_array_equal(a[0].cpu().numpy(), b23[:, ingest.BODY23_TO_21])
    np.testing.assert_array_equal(a[1].cpu().numpy(), l20[:, ingest.HAND_ORDER])
    np.testing.assert_array_equal(a[2].cpu().numpy(), r20[:, ingest.HAND_ORDER])
    np.testing.assert_array_equal(a[3].cpu().numpy(), ~np.array([np.allclose(x, 0) for x in b23]))


@pytest.mark.parametrize("layout", ["aos", "soa"])
def test_solver_full_size_properties(gpu, layout):
    """BASELINE config 3 size (262144 frames, device-generated) in both input layouts -- SoA is the bench
    headline: finite, zero DOFs where the reference never writes, gripper range, and a 2048-frame sample
    identical to the oracle, bit for bit."""
    import oracle as orc
    from rtg import _lib, ops
    zp = golden("zero_pose")
    T = _topo("vtrdyn_full")
    B = 262144
    body, lh, rh = ops.synth_full_body(T, B, seed=99)
    S = _solver(_lib.SOLVER_FULL_BODY_POS, True)
    if layout == "soa":
        sb, sl, sr = ops.synth_full_body(T, B, seed=99, layout="soa")
        assert torch.equal(body.permute(1, 2, 0), sb)
        dof, _, _ = S.retarget([sb, sl, sr], layout="soa")
    else:
        dof, _, _ = S.retarget([body, lh, rh])
    dof_np = _np(dof)
    assert np.isfinite(dof_np).all()
    np.testing.assert_array_equal(dof_np[:, list(range(11)) + [29]], 0.0)
    assert (dof_np[:, [18, 27]] >= 0).all() and (dof_np[:, [18, 27]] <= np.float32(0.044)).all()
    np.testing.assert_array_equal(dof_np[:, 19], -dof_np[:, 18])
    idx = np.random.default_rng(0).choice(B, 2048, replace=False)
    odof, _, _ = orc.full_body_pos(zp["vtrdyn_full_local_t"], zp["vtrdyn_full_global_t"], _np(body)[idx],
                                   _np(lh)[idx], _np(rh)[idx], True, want_rot=False)
    np.testing.assert_array_equal(dof_np[idx], odof)
    # determinism: a second launch is bit-identical
    dof2, _, _ = S.retarget([sb, sl, sr], layout="soa") if layout == "soa" else S.retarget([body, lh, rh])
    assert torch.equal(dof, dof2)


def test_motion_velocities_vs_oracle(gpu):
    import oracle as orc
    from rtg import ops
    m = golden("motion")
    w, _ = ops.gaussian_taps()
    np.testing.assert_array_equal(_np(ops.motion_velocity(m["global_pos"], 1 / 30)), m["global_velocity"])
    av = _np(ops.motion_angular_velocity(m["global_rot"], 1 / 30))
    np.testing.assert_array_equal(av, orc.angular_velocity(m["global_rot"], 1 / 30, w))
    # unsmoothed variant and batched sequences
    lv = _np(ops.motion_velocity(np.stack([m["global_pos"]] * 3), 1 / 30, smooth=False))
    np.testing.assert_array_equal(lv[1], orc.linear_velocity(m["global_pos"], 1 / 30, None))


@pytest.mark.parametrize("nseq,L,J", [(1, 2, 1), (5, 37, 3), (3, 41, 31), (2, 19, 100), (7, 300, 24), (8, 130, 31),
                                     (2, 40, 200)])
def test_motion_velocities_row_tiles(gpu, nseq, L, J):
    """The velocity kernels across tile shapes -- bit-exact against the oracle, smoothed and raw.  Smoothed: the
    one-pass frame-tile kernel with 64-frame tiles, 16-frame tiles (J=100: 300 channels per row), block counts
    that are and are not multiples of 8 (the XCD order), sequences shorter than the filter radius (L=2) and the
    two-pass fallback for rows too wide for LDS (J=200).  Raw: the row-tiled kernels, rows that do not fill a
    block, channel counts that are not powers of two, rows wider than 256 channels (gridDim.y slices)."""
    import oracle as orc
    from rtg import ops
    g = np.random.default_rng(nseq * 1000 + L + J)
    p = g.standard_normal((nseq, L, J, 3)).astype(np.float32)
    q = g.standard_normal((nseq, L, J, 4)).astype(np.float32)
    q /= np.linalg.norm(q, axis=-1, keepdims=True)
    w, _ = ops.gaussian_taps()
    np.testing.assert_array_equal(_np(ops.motion_velocity(p, 1 / 30)), orc.linear_velocity(p, 1 / 30, w))
    np.testing.assert_array_equal(_np(ops.motion_velocity(p, 1 / 30, smooth=False)),
                                  orc.linear_velocity(p, 1 / 30, None))
    np.testing.assert_array_equal(_np(ops.motion_angular_velocity(q, 1 / 30)), orc.angular_velocity(q, 1 / 30, w))
    np.testing.assert_array_equal(_np(ops.motion_angular_velocity(q, 1 / 30, smooth=False)),
                                  orc.angular_velocity(q, 1 / 30, None))


@pytest.mark.parametrize("sigma", [0.1, 0.2, 1.0, 3.5])
def test_motion_velocities_other_filter_radii(gpu, sigma):
    """Filters other than the reference's sigma 2 (radius 0, 1, 4, 14) take the one-pass kernel's generic-radius
    branch: bit-exact against the oracle with the same taps."""
    import oracle as orc
    from rtg import ops
    g = np.random.default_rng(int(sigma * 10))
    p = g.standard_normal((3, 150, 31, 3)).astype(np.float32)
    q = g.standard_normal((3, 150, 31, 4)).astype(np.float32)
    q /= np.linalg.norm(q, axis=-1, keepdims=True)
    w, radius = ops.gaussian_taps(sigma)
    assert radius == int(4 * sigma + 0.5)
    np.testing.assert_array_equal(_np(ops.motion_velocity(p, 1 / 30, sigma=sigma)), orc.linear_velocity(p, 1 / 30, w))
    np.testing.assert_array_equal(_np(ops.motion_angular_velocity(q, 1 / 30, sigma=sigma)),
                                  orc.angular_velocity(q, 1 / 30, w))

