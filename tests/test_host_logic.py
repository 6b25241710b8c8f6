"""CPU-only: the C ABI loads and exports every symbol rtg.h declares; host-side
validation mirrors the reference's assertions; the drop-in modules import
without a GPU and fail loudly (no CPU fallback) when asked to compute."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO


def _declared_symbols():
    src = open(os.path.join(REPO, "include", "rtg.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char \*)\s*(rtg_\w+)\s*\(", src, flags=re.M)))


def test_library_exports_every_declared_symbol():
    from rtg import _lib
    lib = _lib.lib()
    syms = _declared_symbols()
    assert len(syms) >= 18
    for s in syms:
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, f"{s} has no ctypes signature"
    assert lib.rtg_abi_version() == _lib.ABI_VERSION


def test_topology_validation_before_device_work():
    from rtg import _lib
    lib = _lib.lib()
    h = ctypes.c_void_p()
    fp = ctypes.POINTER(ctypes.c_float)
    ip = ctypes.POINTER(ctypes.c_int32)
    lt = np.zeros((3, 3), np.float32)
    bad = np.array([-1, 2, 0], np.int32)          # parent after child
    rc = lib.rtg_topology_create(bad.ctypes.data_as(ip), lt.ctypes.data_as(fp), None, 3, ctypes.byref(h))
    assert rc == 1 and b"parents[1]" in lib.rtg_last_error()
    noroot = np.array([0, 0, 1], np.int32)
    assert lib.rtg_topology_create(noroot.ctypes.data_as(ip), lt.ctypes.data_as(fp), None, 3, ctypes.byref(h)) == 1


def test_solver_and_op_validation():
    from rtg import _lib
    lib = _lib.lib()
    h = ctypes.c_void_p()
    fp = ctypes.POINTER(ctypes.c_float)
    zl = np.zeros((21, 3), np.float32)
    assert lib.rtg_solver_create(0, zl.ctypes.data_as(fp), zl.ctypes.data_as(fp), None, 21, 0, ctypes.byref(h)) == 1
    assert b"59-joint" in lib.rtg_last_error()
    assert lib.rtg_solver_create(9, zl.ctypes.data_as(fp), None, None, 21, 0, ctypes.byref(h)) == 1
    assert lib.rtg_quat_in_xyz_axis_f32(None, b"XyZ", 1, None, None) == 1          # mixed case
    assert lib.rtg_quat_in_xyz_axis_f32(None, b"XXZ", 1, None, None) == 1          # repeated axis
    assert lib.rtg_quat_op_f32(99, None, None, None, 1, None, None) == 1
    assert lib.rtg_cal_joint_quat_f32(None, None, 9, 1, None, None) == 4
    assert lib.rtg_retarget_f32(None, None, None, None, None, 1, 0, None, None, None, None) == 1
    assert lib.rtg_frame_server_launch(None, None, None, None, None, None, 200, None) == 1
    assert b"NULL solver" in lib.rtg_last_error()


def test_dof_model_validation():
    from rtg import _lib
    lib = _lib.lib()
    h = ctypes.c_void_p()
    ax = np.zeros(4, np.int32)
    ip = ctypes.POINTER(ctypes.c_int32)
    assert lib.rtg_dof_model_create(None, ax.ctypes.data_as(ip), None, None, ctypes.byref(h)) == 1
    assert b"NULL topology" in lib.rtg_last_error()
    assert lib.rtg_dof_fk_f32(None, None, None, None, 1, 0, None, None, None) == 1


def test_empty_batches_are_noops():
    from rtg import _lib
    lib = _lib.lib()
    assert lib.rtg_quat_op_f32(0, None, None, None, 0, None, None) == 0
    assert lib.rtg_cal_joint_quat_f32(None, None, 3, 0, None, None) == 0


def test_dropin_modules_import_without_gpu():
    import poselib.poselib.core.rotation3d  # noqa: F401
    import poselib.poselib.skeleton.skeleton3d  # noqa: F401
    import retarget.retarget_solver  # noqa: F401
    import retarget.spatial_transform.transform3d  # noqa: F401
    import robot_kinematics_model  # noqa: F401
    from retarget.retarget_solver import VtrdynFullBodyPosRetargeter  # noqa: F401
    from robot_kinematics_model.hu_forward_model import HuForwardModel  # noqa: F401
    from retarget.main import Retarget, RetargetHuV5fromMocap  # noqa: F401


@pytest.mark.skipif(__import__("torch").cuda.is_available(), reason="checks the no-GPU behaviour")
def test_compute_without_gpu_fails_loudly():
    import torch
    from poselib.poselib.core.rotation3d import quat_mul
    with pytest.raises(RuntimeError, match="no HIP device"):
        quat_mul(torch.zeros(1, 4), torch.zeros(1, 4))


def test_safe_pickle_reader_roundtrip(tmp_path):
    """rtg.safe_pickle decodes a SkeletonState pickle (our own file) without unpickling."""
    import pickle
    import torch
    from poselib.poselib.skeleton.skeleton3d import SkeletonState, SkeletonTree
    from rtg.safe_pickle import load_skeleton_state_arrays
    from rtg import assets
    tree = SkeletonTree([str(s) for s in assets.load("vtrdyn")["node_names"]], torch.from_numpy(assets.parents("vtrdyn")),
                        torch.from_numpy(assets.local_translation("vtrdyn")))
    st = SkeletonState(torch.from_numpy(assets.load("vtrdyn")["tensor"]), tree, True)
    st.__class__.__module__ = "poselib.poselib.skeleton.skeleton3d"
    p = tmp_path / "state.pkl"
    with open(p, "wb") as f:
        pickle.dump(st, f, protocol=4)
    d = load_skeleton_state_arrays(str(p))
    np.testing.assert_array_equal(d["local_translation"], assets.local_translation("vtrdyn"))
    np.testing.assert_array_equal(d["parent_indices"], assets.parents("vtrdyn"))
    assert d["node_names"] == [str(s) for s in assets.load("vtrdyn")["node_names"]]


def test_synthetic_generator_deterministic():
    from rtg import synth
    a = synth.synth_full_body_inputs(8, 5)
    b = synth.synth_full_body_inputs(8, 5)
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)
    assert a[0].shape == (8, 21, 3) and a[1].shape == (8, 20, 3) and a[0].dtype == np.float32


def _fake_solver(kind):
    """A Solver shell (no device handle) to exercise the host-side argument checks without a GPU."""
    import torch
    from rtg.runtime import Solver
    s = Solver.__new__(Solver)
    s._h, s.kind, s.precise_gripper, s.device = None, kind, True, torch.device("cuda", 0)
    return s


def test_solver_rejects_bad_input_shapes():
    """trailing shapes are checked against the kind's rows before anything reaches the C ABI (which
    cannot see shapes): a raw (B,23,3) broadcast body, short hands, mismatched batches, a bad layout."""
    import torch
    from rtg import _lib
    s = _fake_solver(_lib.SOLVER_FULL_BODY_POS)
    B = 4
    good = [torch.zeros(B, 21, 3), torch.zeros(B, 20, 3), torch.zeros(B, 20, 3)]
    cases = [
        [torch.zeros(B, 23, 3), good[1], good[2]],           # raw 23-joint broadcast body
        [good[0], torch.zeros(B, 19, 3), good[2]],            # short hand
        [good[0], good[1], torch.zeros(B + 1, 20, 3)],        # batch mismatch
        [good[0], good[1]],                                   # missing input
    ]
    for ins in cases:
        with pytest.raises(ValueError):
            s.retarget(ins)
    with pytest.raises(ValueError):
        s.retarget(good, layout="planar")
    with pytest.raises(ValueError):   # AoS tensors handed over as SoA
        s.retarget(good, layout="soa")
    with pytest.raises(ValueError):   # CPU tensors of the right shape: not device tensors
        s.retarget(good)
    r = _fake_solver(_lib.SOLVER_FULL_BODY_ROT)
    with pytest.raises(ValueError):   # rotations need 4 components
        r.retarget([torch.zeros(B, 21, 3), torch.zeros(B, 21, 3), torch.zeros(B, 20, 3), torch.zeros(B, 20, 3)])
