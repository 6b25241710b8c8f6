"""VTRDyn ingest: the data formats in front of the retarget solver.

* Socket frames (mocap_communication/mocap_receiver.py:21-26, 49-59): a 4-byte
  big-endian length, then a pickled ``dict`` of float32 arrays ``body_pos``
  (23,3), ``body_quat`` (23,4), ``left_hand_pos`` / ``right_hand_pos`` (20,3).
  The reference ``pickle.loads`` the network bytes, which runs whatever the
  sender names.  :func:`decode_frame` walks the opcodes instead
  (:mod:`rtg.safe_pickle`) and rebuilds arrays only through numpy's own
  reconstructors, from raw bytes; any other callable is rejected.
* CSV recordings (retarget/utils/parse_mocap.py:26-62): one column per joint
  and axis, ``"{joint} position X(m)"`` / ``"{joint} quaternion X"``.
* Reindexing (sim_full_body_teleop.py:109-112): the 23-joint broadcast body to
  the 21-joint VTRDYN order, the 20-point hands to the solver's order.  Batches
  are gathered on the device (``rtg_ingest_vtrdyn_f32``), which also flags the
  frames the teleop loop skips (``np.allclose(body_pos, 0)``, :92).
"""
from __future__ import annotations

import io
import pickle
import struct
from typing import Any, Dict, Optional

import numpy as np
import torch

from ._lib import LAYOUT_SOA, check, lib
from .runtime import dev_f32, layout_code, ptr, stream_handle
from .safe_pickle import Call, Global, Obj, _run_vm

# sim_full_body_teleop.py:109 (23 -> 21) and :111-112 (hand point order)
BODY23_TO_21 = [0, 1, 2, 3, 5, 6, 7, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20, 21, 22]
HAND_ORDER = [0, 4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 12, 13, 14, 15, 1, 2, 3]
FRAME_KEYS = {"body_pos": (23, 3), "body_quat": (23, 4), "left_hand_pos": (20, 3), "right_hand_pos": (20, 3)}

_RECONSTRUCT = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct")}
_FROMBUFFER = {("numpy.core.numeric", "_frombuffer"), ("numpy._core.numeric", "_frombuffer")}
_SCALAR = {("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar")}


def _is(g: Any, names) -> bool:
    return isinstance(g, Global) and (g.module, g.name) in names


def _dtype(node: Any) -> np.dtype:
    """numpy.dtype(code, align, copy) + its BUILD state (version, byte order, ...)."""
    if not (isinstance(node, Call) and _is(node.func, {("numpy", "dtype")})):
        raise ValueError("expected a numpy dtype record")
    dt = np.dtype(str(node.args[0]))
    st = node.state
    if isinstance(st, tuple) and len(st) > 1 and st[1] in ("<", ">"):
        dt = dt.newbyteorder(st[1])
    if dt.hasobject:
        raise ValueError("object arrays are not accepted")
    return dt


def _value(node: Any) -> Any:
    """Inert tree -> Python / numpy values; only numpy array / scalar reconstructors are honoured."""
    if isinstance(node, dict):
        return {_value(k): _value(v) for k, v in node.items()}
    if isinstance(node, list):
        return [_value(v) for v in node]
    if isinstance(node, tuple):
        return tuple(_value(v) for v in node)
    if isinstance(node, (str, int, float, bool, bytes, type(None))):
        return node
    if isinstance(node, bytearray):
        return bytes(node)
    if isinstance(node, Call):
        if _is(node.func, _RECONSTRUCT):   # protocol <= 4: _reconstruct(ndarray, (0,), b'b') + __setstate__
            _ver, shape, dt, fortran, raw = node.state
            raw = _value(raw)
            a = np.frombuffer(raw, dtype=_dtype(dt)).reshape(tuple(shape), order="F" if fortran else "C")
            return a.copy()
        if _is(node.func, _FROMBUFFER):    # protocol 5, in-band buffer
            buf, dt, shape, order = node.args
            return np.frombuffer(bytes(buf), dtype=_dtype(dt)).reshape(tuple(shape), order=order).copy()
        if _is(node.func, _SCALAR):
            dt, raw = node.args
            return np.frombuffer(_value(raw), dtype=_dtype(dt))[0]
        if _is(node.func, {("_codecs", "encode")}) and len(node.args) == 2 and node.args[1] == "latin1":
            return str(node.args[0]).encode("latin1")   # protocol 2 spelling of bytes
        raise ValueError(f"refusing to call {getattr(node.func, 'qualname', node.func)!r} from a mocap frame")
    if isinstance(node, Obj):
        raise ValueError("refusing to instantiate objects from a mocap frame")
    raise ValueError(f"unsupported value {type(node).__name__} in a mocap frame")


def decode_frame(payload: bytes) -> Dict[str, np.ndarray]:
    """One frame payload (the bytes after the length prefix) -> dict of float32 arrays, executing nothing."""
    d = _value(_run_vm(io.BytesIO(payload)))
    if not isinstance(d, dict):
        raise ValueError("mocap frame is not a dict")
    out = {}
    for k, shape in FRAME_KEYS.items():
        if k in d:
            a = np.asarray(d[k], dtype=np.float32)
            if a.shape != shape:
                raise ValueError(f"{k}: expected {shape}, got {a.shape}")
            out[k] = a
    return out


def encode_frame(frame: Dict[str, np.ndarray]) -> bytes:
    """The sender side: 4-byte big-endian length + pickled dict (mocap_receiver.py:49-59)."""
    body = pickle.dumps({k: np.ascontiguousarray(v, dtype=np.float32) for k, v in frame.items()})
    return struct.pack(">I", len(body)) + body


def read_frame(sock) -> Optional[Dict[str, np.ndarray]]:
    """Read one length-prefixed frame from a connected stream socket; None when the peer closed."""
    def recv_n(n):
        data = b""
        while len(data) < n:
            pkt = sock.recv(n - len(data))
            if not pkt:
                return None
            data += pkt
        return data

    hdr = recv_n(4)
    if hdr is None:
        return None
    body = recv_n(int.from_bytes(hdr, "big"))
    return None if body is None else decode_frame(body)


# ---------------------------------------------------------------- CSV recordings (parse_mocap.py:26-62)
def _columns(df, names, fields) -> np.ndarray:
    out = np.zeros((len(df), len(names), len(fields)))        # float64, as the reference
    for j, name in enumerate(names):
        for c, field in enumerate(fields):
            out[:, j, c] = df[f"{name} {field}"]
    return out


_POS = ("position X(m)", "position Y(m)", "position Z(m)")
_QUAT = ("quaternion X", "quaternion Y", "quaternion Z", "quaternion W")


def get_vtrdyn_translation(df) -> np.ndarray:
    from retarget.robot_config import VTRDYN
    return _columns(df, VTRDYN.VTRDYN_JOINT_NAMES, _POS)


def get_vtrdyn_rotation(df) -> np.ndarray:
    from retarget.robot_config import VTRDYN
    return _columns(df, VTRDYN.VTRDYN_JOINT_NAMES, _QUAT)


def get_vtrdyn_full_translation(df) -> np.ndarray:
    from retarget.robot_config import VTRDYN_FULL
    return _columns(df, VTRDYN_FULL.VTRDYN_JOINT_NAMES, _POS)


def get_vtrdyn_full_rotation(df) -> np.ndarray:
    from retarget.robot_config import VTRDYN_FULL
    return _columns(df, VTRDYN_FULL.VTRDYN_JOINT_NAMES, _QUAT)


# ---------------------------------------------------------------- batched device reindex
def reindex_frames(body23, left20, right20, layout="aos"):
    """(B,23,3), (B,20,3), (B,20,3) raw broadcast frames -> solver inputs (B,21,3), (B,20,3), (B,20,3) and a
    (B,) bool "frame carries data" flag (not np.allclose(body_pos, 0)), gathered on the device.  ``layout="soa"``
    emits the solver inputs as component planes (21,3,B), (20,3,B), (20,3,B) directly (rtg.h rtg_layout)."""
    b = dev_f32(body23, (23, 3), "body_pos")
    lh = dev_f32(left20, (20, 3), "left_hand_pos")
    rh = dev_f32(right20, (20, 3), "right_hand_pos")
    B = int(b.shape[0])
    if lh.shape[0] != B or rh.shape[0] != B:
        raise ValueError("frame batches differ in length")
    code = layout_code(layout)
    soa = code == LAYOUT_SOA
    ob = torch.empty((21, 3, B) if soa else (B, 21, 3), device=b.device, dtype=torch.float32)
    ol = torch.empty((20, 3, B) if soa else (B, 20, 3), device=b.device, dtype=torch.float32)
    orr = torch.empty((20, 3, B) if soa else (B, 20, 3), device=b.device, dtype=torch.float32)
    valid = torch.empty((B,), device=b.device, dtype=torch.uint8)
    check(lib().rtg_ingest_vtrdyn_f32(ptr(b), ptr(lh), ptr(rh), B, code, ptr(ob), ptr(ol), ptr(orr), ptr(valid),
                                      stream_handle()))
    return ob, ol, orr, valid.bool()


def hold_last_valid(dof: torch.Tensor, valid: torch.Tensor, last: Optional[torch.Tensor] = None) -> torch.Tensor:
    """The teleop loop's fallback (sim_full_body_teleop.py:92, 121-123): a frame without data repeats the
    previous frame's DOFs (``last`` before the first one; zeros by default, :86)."""
    B = dof.shape[0]
    idx = torch.where(valid, torch.arange(B, device=dof.device), torch.full((B,), -1, device=dof.device))
    src = torch.cummax(idx, dim=0).values
    prev = torch.zeros_like(dof[0]) if last is None else last.to(dof.device, dof.dtype)
    return torch.where((src >= 0).unsqueeze(-1), dof[src.clamp(min=0)], prev.expand_as(dof))


def stack_frames(frames) -> Dict[str, np.ndarray]:
    """List of decoded frames -> contiguous (B, ...) host arrays (pin them for asynchronous H2D copies)."""
    return {k: np.stack([f[k] for f in frames]).astype(np.float32) for k in ("body_pos", "left_hand_pos",
                                                                             "right_hand_pos")}


__all__ = ["BODY23_TO_21", "HAND_ORDER", "decode_frame", "encode_frame", "read_frame", "get_vtrdyn_translation",
           "get_vtrdyn_rotation", "get_vtrdyn_full_translation", "get_vtrdyn_full_rotation", "reindex_frames",
           "hold_last_valid", "stack_frames"]
