"""Degenerate frames on the GPU: the frames the reference raises on, and the ones it solves anyway.

The fixtures (tools/make_golden.py *_edge) hold, per frame, the reference's outputs or the exception it raised:
RuntimeError from torch.linalg.svd on a NaN Kabsch matrix (transform3d.py:40) or ValueError from scipy's from_quat
on a zero / NaN quaternion (transform3d.py:53).  The batched kernels mark such frames (rtg.h rtg_frame_error:
every dof NaN, the code in dof[f, 0]'s payload, local_rot / body_rot rows NaN); the drop-in per-frame calls raise
the reference's exception.  Every comparison with the oracle is on the raw bits (every NaN reading alike, see _bits;
the frame codes compared exactly), through each kernel that serves FULL_BODY_POS: k_fbp_frame1 (B = 1), k_fbp_quad (B <= RTG_QUAD_MAX_B: the fixture
as one batch), k_fbp_latency5 (B <= RTG_LATENCY_MAX_B) and k_solve_sides (larger; edge frames scattered through
ragged batches whose last tile is partly empty)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

from conftest import PKG, REPO, golden

pytestmark = pytest.mark.gpu

EXC = {1: (RuntimeError, "linalg.svd: \\(Batch element 0\\): The algorithm failed to converge because the input "
                         "matrix contained non-finite values."),
       2: (ValueError, "Found zero norm quaternions in `quat`.")}


def _bits(a):
    """The raw float32 bits -- except that every NaN reads as one value: the sign and payload of a NaN that
    arithmetic produced or propagated differ between x86 (the oracle) and the GPU and carry no meaning.  The
    frame-status payloads (dof[f, 0]) are compared separately, bit for bit, through frame_status."""
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    a = np.ascontiguousarray(a, np.float32)
    return np.where(np.isnan(a), np.uint32(0x7FC00000), a.view(np.uint32))


def _solver(kind, precise=False):
    from rtg import _lib, assets
    from rtg.runtime import Solver
    zp = golden("zero_pose")
    if kind in (_lib.SOLVER_FULL_BODY_POS, _lib.SOLVER_FULL_BODY_ROT):
        return Solver(kind, zp["vtrdyn_full_local_t"], zp["vtrdyn_full_global_t"], assets.parents("vtrdyn_full"),
                      precise)
    return Solver(kind, zp["vtrdyn_local_t"], zp["vtrdyn_global_t"], assets.parents("vtrdyn"), precise)


CASES = [("full_body_pos_edge", 0, True), ("full_body_pos_edge", 0, False), ("upper_body_edge", 1, False),
         ("full_body_rot_edge", 2, False), ("body_rot_edge", 3, False)]
INPUTS = {0: ("body", "lh", "rh"), 1: ("x",), 2: ("body_rot", "body_pos", "lh", "rh"), 3: ("global_rot",)}


def _oracle(kind, d, precise):
    import oracle as orc
    from rtg import assets
    zp = golden("zero_pose")
    if kind == 0:
        return orc.full_body_pos(zp["vtrdyn_full_local_t"], zp["vtrdyn_full_global_t"], d["body"], d["lh"], d["rh"],
                                 precise)
    if kind == 1:
        return orc.upper_body(zp["vtrdyn_local_t"], d["x"]) + (None,)
    if kind == 2:
        return orc.full_body_rot(zp["vtrdyn_full_local_t"], d["body_rot"], d["body_pos"], d["lh"], d["rh"]) + (None,)
    return orc.body_rot(assets.parents("vtrdyn"), d["global_rot"]) + (None,)


def _ref_status(name, d, precise):
    if name == "full_body_pos_edge":
        return d["precise_status" if precise else "binary_status"]
    return d["status"]


@pytest.mark.parametrize("name,kind,precise", CASES)
def test_edge_frames_gpu_equals_oracle_every_kernel(gpu, name, kind, precise):
    from rtg.runtime import frame_status
    d = golden(name)
    ins = [torch.from_numpy(np.ascontiguousarray(d[k])).cuda() for k in INPUTS[kind]]
    n = ins[0].shape[0]
    odof, olr, obr = _oracle(kind, d, precise)
    S = _solver(kind, precise)
    fbp = kind == 0
    # the whole fixture as one batch (k_fbp_quad for FULL_BODY_POS, k_solve_sides otherwise)
    dof, lr, br = S.retarget(ins, want_local_rot=True, want_body_rot=fbp)
    import oracle as orc
    np.testing.assert_array_equal(orc.frame_status(odof), _ref_status(name, d, precise))
    np.testing.assert_array_equal(_bits(dof), _bits(odof))
    np.testing.assert_array_equal(_bits(lr), _bits(olr))
    if fbp:
        np.testing.assert_array_equal(_bits(br), _bits(obr))
    np.testing.assert_array_equal(frame_status(dof).cpu().numpy(), _ref_status(name, d, precise))
    # SoA inputs, same bits
    dof_s, lr_s, _ = S.retarget([t.permute(1, 2, 0).contiguous() for t in ins], want_local_rot=True, layout="soa")
    np.testing.assert_array_equal(_bits(dof_s), _bits(odof))
    np.testing.assert_array_equal(frame_status(dof_s).cpu().numpy(), _ref_status(name, d, precise))
    np.testing.assert_array_equal(_bits(lr_s), _bits(olr))
    # scattered through ragged larger batches: k_solve_sides (65536 + 40 leaves the last block's second tile empty)
    # and, for FULL_BODY_POS, k_fbp_latency5 (a size between the build's quad and latency bounds, 64-frame tiles)
    from rtg import _lib
    info = _lib.build_info()["knobs"]
    sizes = [65536 + 40]
    if fbp and info["RTG_QUAD_MAX_B"] + 40 <= info["RTG_LATENCY_MAX_B"]:
        sizes.append(info["RTG_QUAD_MAX_B"] + 40)
    for B in sizes:
        g = torch.Generator().manual_seed(5)
        idx = torch.randint(0, n, (B,), generator=g)
        idx[-n:] = torch.arange(n)   # every edge frame, including in the last, partly empty block
        big = [t[idx.cuda()].contiguous() for t in ins]
        dof_b, lr_b, br_b = S.retarget(big, want_local_rot=True, want_body_rot=fbp)
        sel = idx.numpy()
        np.testing.assert_array_equal(frame_status(dof_b).cpu().numpy(), _ref_status(name, d, precise)[sel])
        np.testing.assert_array_equal(_bits(dof_b), _bits(odof)[sel])
        np.testing.assert_array_equal(_bits(lr_b), _bits(olr)[sel])
        if fbp:
            np.testing.assert_array_equal(_bits(br_b), _bits(obr)[sel])
    if fbp:
        # one frame per launch (k_fbp_frame1)
        for i in range(n):
            d1, l1, b1 = S.retarget([t[i:i + 1] for t in ins], want_local_rot=True, want_body_rot=True)
            np.testing.assert_array_equal(_bits(d1), _bits(odof[i:i + 1]))
            assert frame_status(d1).item() == _ref_status(name, d, precise)[i]
            np.testing.assert_array_equal(_bits(l1), _bits(olr[i:i + 1]))
            np.testing.assert_array_equal(_bits(b1), _bits(obr[i:i + 1]))


@pytest.fixture(scope="module")
def poses(gpu):
    from robot_kinematics_model import RobotZeroPose
    return {n: RobotZeroPose.from_asset(n) for n in ("hu_v5", "vtrdyn_full", "vtrdyn")}


@pytest.mark.parametrize("server", [False, True])
def test_dropin_retarget_raises_like_the_reference(poses, server):
    """sim_full_body_teleop.py:115-119's per-frame call: a frame the reference raises on raises the same exception
    type and message (and records nothing); the other frames return the oracle's values, NaNs included."""
    import oracle as orc
    from retarget.retarget_solver import VtrdynFullBodyPosRetargeter
    d = golden("full_body_pos_edge")
    odof, olr, obr = _oracle(0, d, True)
    s = VtrdynFullBodyPosRetargeter(poses["vtrdyn_full"], poses["hu_v5"], precise_gripper=True, frame_server=server,
                                    idle_ms=50)
    try:
        status = d["precise_status"]
        for i in range(len(status)):
            args = [torch.from_numpy(d[k][i]) for k in ("body", "lh", "rh")]
            before = s.motion_length
            if status[i]:
                exc, msg = EXC[int(status[i])]
                with pytest.raises(exc, match=msg):
                    s.retarget(*args)
                assert s.motion_length == before
            else:   # every output, including the rows the server writes only once (a raising frame before
                lr, dof, br = s.retarget(*args)   # overwrote them with NaN: they must be back)
                np.testing.assert_array_equal(_bits(dof), _bits(odof[i]))
                np.testing.assert_array_equal(_bits(lr), _bits(olr[i]))
                np.testing.assert_array_equal(_bits(br), _bits(obr[i]))
                assert s.motion_length == before + 1
        assert s.motion_length == int(d["precise_recorded"])   # the reference recorded exactly these frames
        assert orc.frame_status(odof).tolist() == status.tolist()
    finally:
        s.close()


@pytest.mark.parametrize("name,kind", [("upper_body_edge", 1), ("full_body_rot_edge", 2), ("body_rot_edge", 3)])
def test_dropin_other_solvers_raise_like_the_reference(poses, name, kind):
    from retarget.retarget_solver import (HuUpperBodyFromMocapRetarget, Mocap2HuBodyRetargeter,
                                          VtrdynFullBodyRetargeter)
    d = golden(name)
    status = d["status"]
    odof, _, _ = _oracle(kind, d, False)
    if kind == 1:
        s = HuUpperBodyFromMocapRetarget(poses["vtrdyn"], poses["hu_v5"])
        call = lambda i: s.retarget_from_global_translation(torch.from_numpy(d["x"][i]))   # noqa: E731
    elif kind == 2:
        s = VtrdynFullBodyRetargeter(poses["vtrdyn_full"], poses["hu_v5"])
        call = lambda i: s.retarget(*[torch.from_numpy(d[k][i]) if k else None   # noqa: E731
                                      for k in ("body_rot", "body_pos", None, "lh", None, "rh")])
    else:
        s = Mocap2HuBodyRetargeter(poses["vtrdyn"], poses["hu_v5"])
        call = lambda i: s.retarget_from_pose(torch.from_numpy(d["global_rot"][i]))   # noqa: E731
    for i in range(len(status)):
        if status[i]:
            exc, msg = EXC[int(status[i])]
            with pytest.raises(exc, match=msg):
                call(i)
        else:
            _, dof = call(i)
            np.testing.assert_array_equal(_bits(dof), _bits(odof[i]))
    assert s.motion_length == int((status == 0).sum())
    # on the device the per-frame call raises too (the batched path at B = 1)
    i = int(np.argmax(status != 0))
    if kind == 1:
        with pytest.raises(EXC[int(status[i])][0]):
            s.retarget_from_global_translation(torch.from_numpy(d["x"][i]).cuda())


def test_dropin_batch_ok_mask_and_record(poses):
    from retarget.retarget_solver import VtrdynFullBodyPosRetargeter
    d = golden("full_body_pos_edge")
    s = VtrdynFullBodyPosRetargeter(poses["vtrdyn_full"], poses["hu_v5"], precise_gripper=True)
    lr, dof, br, ok = s.retarget_batch(*[torch.from_numpy(d[k]).cuda() for k in ("body", "lh", "rh")],
                                       record=True, return_ok=True)
    np.testing.assert_array_equal(ok.cpu().numpy(), d["precise_status"] == 0)
    assert torch.isnan(dof[~ok]).all() and torch.isnan(lr[~ok]).all()
    assert s.motion_length == int(ok.sum())   # only the frames the reference returns a result for are recorded


def test_dropin_primitives_raise_like_the_reference(gpu):
    """transform3d.cal_joint_quat (:31-50), quat_in_xyz_axis (:52-59) and rotation3d.quat_to_eular (:658-661) raise
    where torch.linalg.svd / scipy raise; the rest of the batch is unchanged."""
    from poselib.poselib.core.rotation3d import quat_to_eular
    from retarget.spatial_transform import transform3d as t3
    Z = torch.randn(4, 5, 3)
    M = torch.randn(4, 5, 3)
    q_ok = t3.cal_joint_quat(Z, M)
    assert q_ok.shape == (4, 4) and torch.isfinite(q_ok).all()
    M[2, 1, 0] = float("nan")
    M[3, 0, 2] = float("nan")
    # torch's own error: LinAlgError (a RuntimeError) naming the FIRST non-finite batch element, as eager
    # torch.linalg.svd does on this batch; the per-frame calls name element 0 like the reference
    with pytest.raises(torch.linalg.LinAlgError, match=EXC[1][1].replace("element 0", "element 2")):
        t3.cal_joint_quat(Z, M)
    A = torch.einsum("bij,bjk->bik", M.permute(0, 2, 1), Z)
    with pytest.raises(torch.linalg.LinAlgError, match="Batch element 2"):
        torch.linalg.svd(A)
    q = torch.nn.functional.normalize(torch.randn(3, 4), dim=-1)
    t3.quat_in_xyz_axis(q, "XYZ")
    q[1] = 0.0
    with pytest.raises(EXC[2][0], match=EXC[2][1]):
        t3.quat_in_xyz_axis(q, "XYZ")
    with pytest.raises(EXC[2][0], match=EXC[2][1]):
        quat_to_eular(q)
    q[1] = torch.tensor([float("inf"), 0.0, 0.0, 1.0])   # an inf component does not raise in scipy
    t3.quat_in_xyz_axis(q, "XYZ")


SKIP_SIGNAL_LIB = os.path.join(PKG, "variants", "skip_signal.so")
_CHILD = r"""
import sys, numpy as np, torch
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
from conftest import golden
from rtg import _lib, assets, ops
from rtg.runtime import Solver, Topology
zp = golden("zero_pose")
S = Solver(_lib.SOLVER_FULL_BODY_POS, zp["vtrdyn_full_local_t"], zp["vtrdyn_full_global_t"], assets.parents("vtrdyn_full"), True)
T = Topology(assets.parents("vtrdyn_full"), assets.local_translation("vtrdyn_full"), assets.tree_quat("vtrdyn_full"))
b, l, r = ops.synth_full_body(T, 65536 + 40, seed=3)
S.retarget([b, l, r])          # k_solve_sides: block 0's R10 flag never goes up, its right wave times out
torch.cuda.synchronize()
try:
    S.retarget([b, l, r])      # the next call reports it
except _lib.RtgError as e:
    print("REPORTED", e)
    S.retarget([b, l, r])      # reported once, then cleared (this launch times out again, unreported so far)
    torch.cuda.synchronize()
    print("CLEARED")
    sys.exit(0)
print("NOT REPORTED")
sys.exit(1)
"""


def test_handover_timeout_is_reported_not_silent(gpu):
    """A wave whose partner's hand-over flag never arrives gives up after ~0.1 s and ORs
    RTG_DEVERR_HANDOVER_TIMEOUT into the solver's error word; the next rtg_retarget_f32 returns RTG_ERR_DEVICE and the
    binding raises RtgError.  Run once, on the measurement build RTG_EXP_SKIP_SIGNAL=1 (__graft_entry__.build())."""
    if not os.path.exists(SKIP_SIGNAL_LIB):
        pytest.fail(f"{SKIP_SIGNAL_LIB} is missing: build it with __graft_entry__.build()")
    env = dict(os.environ, RTG_LIB=SKIP_SIGNAL_LIB, RTG_ALLOW_MEASUREMENT_BUILD="1")
    r = subprocess.run([sys.executable, "-c", _CHILD, PKG, os.path.join(REPO, "tests")], env=env, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0 and "REPORTED" in r.stdout and "hand-over timed out" in r.stdout, r.stdout + r.stderr
    assert "CLEARED" in r.stdout


@pytest.mark.gpu
def test_bench_device_path_two_ranks_on_one_gpu():
    """bench.py's N>1 DEVICE flow rehearsed on the one-GPU box: two rank processes on cuda:0 (gloo collectives,
    tests/bench_shared_gpu_backend.py), each with its two streams, clock settle and single-launch kernel time.  Rank 0
    prints the line with n_gpus 2, both ranks pass their golden check, and the gathered DOFs hold both shards."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(RTG_BENCH_BACKEND="bench_shared_gpu_backend:SharedGpuGlooBackend", RTG_BENCH_SETTLE_MS="20",
               PYTHONPATH=os.pathsep.join([os.path.dirname(os.path.abspath(__file__)), repo, env.get("PYTHONPATH", "")]))
    r = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2", "--steps", "6", "--warmup", "2",
                        "--batch", "65536", "--no-cpu-baseline"], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "dp2"
    assert line["value"] > 0 and line["roofline"]["kernel_ms"] > 0 and line["settle"]["blocks_of_K_steps"] >= 1
    assert [g["rank"] for g in line["golden_per_rank"]] == [0, 1]
    assert all(g["max_abs_err"] < 1e-4 for g in line["golden_per_rank"])
    assert "gather_ms" in line
    # both ranks report the device they ran on (the same card here: the rehearsal backend sets SHARES_DEVICE) and the
    # line names the collective backend and the RCCL build torch carries
    assert [d["rank"] for d in line["devices"]] == [0, 1] and all(d["pci"] for d in line["devices"])
    assert line["comm"]["backend"] == "gloo" and line["comm"]["rccl_version"]


_BAD_STREAM_CHILD = r"""
import ctypes, sys, numpy as np, torch
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[2])
from conftest import golden
from rtg import _lib, assets, ops
from rtg._lib import lib
from rtg.runtime import Solver, Topology, ptr
zp = golden("zero_pose")
S = Solver(_lib.SOLVER_FULL_BODY_POS, zp["vtrdyn_full_local_t"], zp["vtrdyn_full_global_t"], assets.parents("vtrdyn_full"), True)
T = Topology(assets.parents("vtrdyn_full"), assets.local_translation("vtrdyn_full"), assets.tree_quat("vtrdyn_full"))
hip = ctypes.CDLL("libamdhip64.so")
st = ctypes.c_void_p()
assert hip.hipStreamCreate(ctypes.byref(st)) == 0 and hip.hipStreamDestroy(st) == 0   # a handle HIP no longer knows
for B in (1, 16, 4096, 8192, 65536):   # k_fbp_frame1, k_fbp_quad (8 and 16 frames), k_fbp_latency5, k_solve_sides
    b, l, r = ops.synth_full_body(T, B, seed=5)
    dof = torch.empty((B, 30), device="cuda")
    torch.cuda.synchronize()
    rc = lib().rtg_retarget_f32(S.handle, ptr(b), ptr(l), ptr(r), None, B, _lib.LAYOUT_AOS, ptr(dof), None, None, st.value)
    print("B", B, "rc", rc, lib().rtg_last_error().decode() if rc else "")
    sys.stdout.flush()
"""


def test_failed_launch_is_reported_on_every_kernel(gpu):
    """a launch that fails (here: a stream handle HIP has destroyed) returns a non-OK status from
    rtg_retarget_f32 on every FULL_BODY_POS kernel, the small-batch ones included -- launch_fbp_small reads the error
    state itself, and its result is now passed up instead of a second, already cleared hipGetLastError()."""
    r = subprocess.run([sys.executable, "-c", _BAD_STREAM_CHILD, PKG, os.path.join(REPO, "tests")],
                       capture_output=True, text=True, timeout=120)
    if r.returncode < 0:
        pytest.skip(f"the HIP runtime did not validate the destroyed stream handle (signal {-r.returncode})")
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [x for x in r.stdout.splitlines() if x.startswith("B ")]
    assert len(lines) == 5, r.stdout + r.stderr
    for x in lines:
        assert " rc 0 " not in x + " " and "launch" in x, x
