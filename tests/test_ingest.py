"""VTRDyn ingest: socket frame codec, CSV columns, device reindex + skip flags."""
import pickle
import socket

import numpy as np
import pytest

from conftest import golden


def _frame(rng):
    return {"body_pos": rng.normal(size=(23, 3)).astype(np.float32),
            "body_quat": rng.normal(size=(23, 4)).astype(np.float32),
            "left_hand_pos": rng.normal(size=(20, 3)).astype(np.float32),
            "right_hand_pos": rng.normal(size=(20, 3)).astype(np.float32)}


@pytest.mark.parametrize("proto", [2, 3, 4, 5])
def test_decode_frame_roundtrip(proto):
    from rtg.ingest import decode_frame
    f = _frame(np.random.default_rng(proto))
    got = decode_frame(pickle.dumps(f, protocol=proto))
    assert set(got) == set(f)
    for k in f:
        np.testing.assert_array_equal(got[k], f[k])
        assert got[k].dtype == np.float32


def test_decode_frame_executes_nothing():
    """A payload naming any callable but numpy's array reconstructors is refused, and nothing runs."""
    from rtg.ingest import decode_frame
    hits = []

    class Evil:
        def __reduce__(self):
            return (hits.append, ("ran",))

    with pytest.raises(Exception):
        decode_frame(pickle.dumps({"body_pos": Evil()}))
    payload = pickle.dumps({"body_pos": np.zeros((23, 3), np.float32), "x": Evil()})
    with pytest.raises(ValueError, match="refusing"):
        decode_frame(payload)
    assert hits == []
    with pytest.raises(ValueError):
        decode_frame(pickle.dumps({"body_pos": np.zeros((22, 3), np.float32)}))   # wrong shape


def test_socket_framing():
    """4-byte big-endian length + pickle body (mocap_receiver.py:49-59), read back from a real socket pair."""
    from rtg.ingest import encode_frame, read_frame
    a, b = socket.socketpair()
    try:
        frames = [_frame(np.random.default_rng(i)) for i in range(3)]
        for f in frames:
            a.sendall(encode_frame(f))
        a.shutdown(socket.SHUT_WR)
        for f in frames:
            got = read_frame(b)
            np.testing.assert_array_equal(got["body_pos"], f["body_pos"])
        assert read_frame(b) is None
    finally:
        a.close()
        b.close()


def test_csv_columns():
    """parse_mocap.py:26-62: "{joint} position X(m)" / "{joint} quaternion X" columns -> (L, J, 3|4) float64."""
    import pandas as pd
    from retarget.robot_config import VTRDYN, VTRDYN_FULL
    from rtg.ingest import (get_vtrdyn_full_rotation, get_vtrdyn_full_translation, get_vtrdyn_rotation,
                            get_vtrdyn_translation)
    rng = np.random.default_rng(0)
    for names, fp, fq in ((VTRDYN.VTRDYN_JOINT_NAMES, get_vtrdyn_translation, get_vtrdyn_rotation),
                          (VTRDYN_FULL.VTRDYN_JOINT_NAMES, get_vtrdyn_full_translation, get_vtrdyn_full_rotation)):
        P = rng.normal(size=(7, len(names), 3))
        Qv = rng.normal(size=(7, len(names), 4))
        cols = {}
        for j, n in enumerate(names):
            for c, ax in enumerate("XYZ"):
                cols[f"{n} position {ax}(m)"] = P[:, j, c]
            for c, ax in enumerate("XYZW"):
                cols[f"{n} quaternion {ax}"] = Qv[:, j, c]
        df = pd.DataFrame(cols)
        np.testing.assert_array_equal(fp(df), P)
        np.testing.assert_array_equal(fq(df), Qv)


@pytest.mark.gpu
def test_reindex_and_skip_flags(gpu):
    from rtg.ingest import BODY23_TO_21, HAND_ORDER, reindex_frames
    rng = np.random.default_rng(1)
    B = 3001
    bp = rng.normal(size=(B, 23, 3)).astype(np.float32)
    lh = rng.normal(size=(B, 20, 3)).astype(np.float32)
    rh = rng.normal(size=(B, 20, 3)).astype(np.float32)
    bp[5] = 0.0
    bp[6] = 5e-9                       # allclose(., 0): skipped
    bp[7] = 0.0
    bp[7, 3, 1] = 2e-8                 # one value beyond atol: kept
    bp[8] = 0.0
    bp[8, 0, 0] = np.nan               # NaN is never close: kept
    b, l, r, valid = reindex_frames(bp, lh, rh)
    np.testing.assert_array_equal(b.cpu().numpy(), bp[:, BODY23_TO_21])
    np.testing.assert_array_equal(l.cpu().numpy(), lh[:, HAND_ORDER])
    np.testing.assert_array_equal(r.cpu().numpy(), rh[:, HAND_ORDER])
    want = ~np.array([np.allclose(x, 0) for x in bp])
    np.testing.assert_array_equal(valid.cpu().numpy(), want)


@pytest.mark.gpu
def test_teleop_chain_matches_per_frame_loop(gpu):
    """decode -> stack -> device reindex -> one batched solve -> hold-last == the reference loop structure
    (sim_full_body_teleop.py:86-123) run frame by frame through the drop-in solver."""
    import torch
    from retarget.retarget_solver import VtrdynFullBodyPosRetargeter
    from robot_kinematics_model import RobotZeroPose
    from rtg import _lib, assets
    from rtg.ingest import BODY23_TO_21, HAND_ORDER, decode_frame, encode_frame, hold_last_valid, reindex_frames, stack_frames
    from rtg.runtime import Solver
    g = golden("full_body_pos_precise")
    zp = golden("zero_pose")
    n = 48
    frames = []
    for i in range(n):
        body23 = np.zeros((23, 3), np.float32)
        body23[BODY23_TO_21] = g["body"][i]
        lh = np.zeros((20, 3), np.float32)
        rh = np.zeros((20, 3), np.float32)
        lh[HAND_ORDER] = g["lh"][i]
        rh[HAND_ORDER] = g["rh"][i]
        if i in (3, 4, 20):
            body23[:] = 0.0                        # dropped frames
        frames.append({"body_pos": body23, "body_quat": np.zeros((23, 4), np.float32),
                       "left_hand_pos": lh, "right_hand_pos": rh})
    decoded = [decode_frame(encode_frame(f)[4:]) for f in frames]
    h = stack_frames(decoded)
    b, l, r, valid = reindex_frames(torch.from_numpy(h["body_pos"]).pin_memory(),
                                    torch.from_numpy(h["left_hand_pos"]).pin_memory(),
                                    torch.from_numpy(h["right_hand_pos"]).pin_memory())
    S = Solver(_lib.SOLVER_FULL_BODY_POS, zp["vtrdyn_full_local_t"], zp["vtrdyn_full_global_t"],
               assets.parents("vtrdyn_full"), True)
    dof, _, _ = S.retarget([b, l, r])
    got = hold_last_valid(dof, valid).cpu().numpy()
    # the reference loop, per frame, through the drop-in class
    hu = VtrdynFullBodyPosRetargeter(RobotZeroPose.from_asset("vtrdyn_full"), RobotZeroPose.from_asset("hu_v5"),
                                     precise_gripper=True)
    last = torch.zeros(30)
    want = []
    for f in decoded:
        if not np.allclose(f["body_pos"], 0):
            _, last, _ = hu.retarget(torch.from_numpy(f["body_pos"][BODY23_TO_21]),
                                     torch.from_numpy(f["left_hand_pos"][HAND_ORDER]),
                                     torch.from_numpy(f["right_hand_pos"][HAND_ORDER]))
        want.append(last.cpu().numpy())
    np.testing.assert_array_equal(got, np.stack(want))
