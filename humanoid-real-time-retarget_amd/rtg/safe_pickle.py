"""Non-executing reader for the reference's pickled ``SkeletonState`` assets.

The reference ships its zero poses as ``pickle.dump(SkeletonState)`` files
(``asset/hu_pose/hu_v5_zero_pose.pkl``, ``asset/zero_pose/*.pkl``; produced by
e.g. ``asset/hu_pose/get_hu_pose.py:17-59``).  Loading them with ``pickle.load``
would execute whatever callables the file names.  This module never does that:
it walks the opcode stream with :mod:`pickletools` and interprets only a small,
inert subset of opcodes.  ``GLOBAL``/``STACK_GLOBAL`` become :class:`Global`
markers, ``REDUCE``/``NEWOBJ``/``BUILD`` become plain records, and the only
"calls" ever resolved are the two torch tensor-rebuild helpers, which are
re-implemented here on raw bytes (legacy ``torch.save`` storage layout).

The result is a plain ``dict`` tree of numpy arrays / lists / scalars.
"""
from __future__ import annotations

import io
import pickletools
import struct
from dataclasses import dataclass, field
from typing import Any, Dict, List

import numpy as np

__all__ = ["Global", "Call", "Obj", "PersId", "read_pickle_tree", "read_npy_object", "load_skeleton_state_arrays"]


@dataclass(frozen=True)
class Global:
    module: str
    name: str

    @property
    def qualname(self) -> str:
        return f"{self.module}.{self.name}"


@dataclass
class Call:
    func: Any
    args: Any
    state: Any = None   # BUILD applied to the call's result (numpy arrays: __setstate__ tuple)


@dataclass
class Obj:
    cls: Any
    args: Any
    state: Any = None


@dataclass
class PersId:
    pid: Any


class _Mark:
    pass


_MARK = _Mark()


def _run_vm(stream: io.BytesIO) -> Any:
    """Interpret one pickle (up to STOP) from ``stream`` without executing anything."""
    stack: List[Any] = []
    memo: Dict[int, Any] = {}

    def pop_mark() -> List[Any]:
        items = []
        while True:
            v = stack.pop()
            if v is _MARK:
                break
            items.append(v)
        items.reverse()
        return items

    for op, arg, _pos in pickletools.genops(stream):
        n = op.name
        if n in ("PROTO", "FRAME"):
            continue
        if n == "STOP":
            return stack.pop()
        if n == "MARK":
            stack.append(_MARK)
        elif n == "POP":
            stack.pop()
        elif n == "POP_MARK":
            pop_mark()
        elif n in ("SHORT_BINUNICODE", "BINUNICODE", "BINUNICODE8", "UNICODE",
                   "SHORT_BINSTRING", "BINSTRING", "STRING",
                   "BINBYTES", "SHORT_BINBYTES", "BINBYTES8", "BYTEARRAY8",
                   "BININT", "BININT1", "BININT2", "LONG1", "LONG4", "INT", "LONG",
                   "BINFLOAT", "FLOAT"):
            stack.append(arg)
        elif n == "NONE":
            stack.append(None)
        elif n == "NEWTRUE":
            stack.append(True)
        elif n == "NEWFALSE":
            stack.append(False)
        elif n == "EMPTY_LIST":
            stack.append([])
        elif n == "EMPTY_DICT":
            stack.append({})
        elif n == "EMPTY_TUPLE":
            stack.append(())
        elif n == "APPEND":
            v = stack.pop()
            stack[-1].append(v)
        elif n == "APPENDS":
            items = pop_mark()
            stack[-1].extend(items)
        elif n == "LIST":
            stack.append(pop_mark())
        elif n == "TUPLE":
            stack.append(tuple(pop_mark()))
        elif n == "TUPLE1":
            stack[-1:] = [(stack[-1],)]
        elif n == "TUPLE2":
            stack[-2:] = [tuple(stack[-2:])]
        elif n == "TUPLE3":
            stack[-3:] = [tuple(stack[-3:])]
        elif n == "DICT":
            items = pop_mark()
            stack.append({items[i]: items[i + 1] for i in range(0, len(items), 2)})
        elif n == "SETITEM":
            v = stack.pop()
            k = stack.pop()
            stack[-1][k] = v
        elif n == "SETITEMS":
            items = pop_mark()
            d = stack[-1]
            for i in range(0, len(items), 2):
                d[items[i]] = items[i + 1]
        elif n == "MEMOIZE":
            memo[len(memo)] = stack[-1]
        elif n in ("BINPUT", "LONG_BINPUT", "PUT"):
            memo[int(arg)] = stack[-1]
        elif n in ("BINGET", "LONG_BINGET", "GET"):
            stack.append(memo[int(arg)])
        elif n == "GLOBAL":
            mod, name = arg.split(" ", 1)
            stack.append(Global(mod, name))
        elif n == "STACK_GLOBAL":
            name = stack.pop()
            mod = stack.pop()
            stack.append(Global(mod, name))
        elif n == "REDUCE":
            args = stack.pop()
            func = stack.pop()
            if isinstance(func, Global) and func.qualname == "collections.OrderedDict" and args == ():
                stack.append({})     # an empty mapping that SETITEM(S) fill: plain data, nothing called
            else:
                stack.append(Call(func, args))
        elif n == "NEWOBJ":
            args = stack.pop()
            cls = stack.pop()
            stack.append(Obj(cls, args))
        elif n == "BUILD":
            state = stack.pop()
            target = stack[-1]
            if isinstance(target, (Obj, Call)):
                target.state = state
            else:
                raise ValueError(f"BUILD on unsupported target {type(target)}")
        elif n == "BINPERSID":
            stack.append(PersId(stack.pop()))
        else:
            raise ValueError(f"unsupported pickle opcode {n}")
    raise ValueError("pickle stream ended without STOP")


_STORAGE_DTYPES = {
    "FloatStorage": np.float32,
    "DoubleStorage": np.float64,
    "LongStorage": np.int64,
    "IntStorage": np.int32,
    "ShortStorage": np.int16,
    "CharStorage": np.int8,
    "ByteStorage": np.uint8,
    "BoolStorage": np.bool_,
    "HalfStorage": np.float16,
}


def _legacy_storage_from_bytes(blob: bytes) -> np.ndarray:
    """Decode a legacy ``torch.save`` blob holding exactly one storage.

    Layout (torch ``_legacy_save``): magic pickle, protocol pickle, sys-info
    pickle, object pickle (whose persistent id is
    ``('storage', <Global ...Storage>, key, location, numel, view)``), key-list
    pickle, then per key an ``int64`` element count followed by the raw bytes.
    """
    s = io.BytesIO(blob)
    _magic = _run_vm(s)
    _proto = _run_vm(s)
    _sysinfo = _run_vm(s)
    root = _run_vm(s)
    keys = _run_vm(s)
    if not isinstance(root, PersId):
        raise ValueError("expected a bare storage in the legacy blob")
    tag, stype, key, _loc, numel, _view = root.pid
    if tag != "storage" or not isinstance(stype, Global):
        raise ValueError("unexpected storage persistent id")
    dtype = _STORAGE_DTYPES[stype.name]
    if list(keys) != [key]:
        raise ValueError("multi-storage blobs are not supported")
    (count,) = struct.unpack("<q", s.read(8))
    if count != numel:
        raise ValueError("storage size mismatch")
    raw = s.read(count * np.dtype(dtype).itemsize)
    return np.frombuffer(raw, dtype=dtype).copy()


def _resolve(node: Any) -> Any:
    """Turn the inert record tree into plain python / numpy values."""
    if isinstance(node, Call):
        f = node.func
        if isinstance(f, Global):
            if f.qualname == "torch._utils._rebuild_tensor_v2":
                storage, offset, size, stride = (_resolve(a) for a in node.args[:4])
                itemsize = storage.dtype.itemsize
                arr = np.lib.stride_tricks.as_strided(
                    storage[offset:], shape=tuple(size),
                    strides=tuple(st * itemsize for st in stride))
                return np.array(arr, copy=True)
            if f.qualname == "torch.storage._load_from_bytes":
                return _legacy_storage_from_bytes(node.args[0])
            if f.qualname == "collections.OrderedDict":
                return {}
            if f.qualname in _NP_RECONSTRUCT:          # np.ndarray.__reduce__: rebuilt from its BUILD state
                return _ndarray_from_state(node.state)
            if f.qualname == "numpy.dtype":
                return _dtype_from(node)
            if f.qualname in _NP_SCALAR:
                dt, raw = _resolve(node.args[0]), node.args[1]
                return np.frombuffer(raw, dtype=dt)[0] if dt != np.dtype(object) else raw
        raise ValueError(f"refusing to resolve call to {f}")
    if isinstance(node, Obj):
        cls = node.cls.qualname if isinstance(node.cls, Global) else str(node.cls)
        state = _resolve(node.state) if node.state is not None else {}
        out = {"__class__": cls}
        out.update(state)
        return out
    if isinstance(node, dict):
        return {k: _resolve(v) for k, v in node.items()}
    if isinstance(node, list):
        return [_resolve(v) for v in node]
    if isinstance(node, tuple):
        return tuple(_resolve(v) for v in node)
    return node


_NP_RECONSTRUCT = ("numpy.core.multiarray._reconstruct", "numpy._core.multiarray._reconstruct")
_NP_SCALAR = ("numpy.core.multiarray.scalar", "numpy._core.multiarray.scalar")


def _dtype_from(node: Call) -> np.dtype:
    """numpy.dtype('<code>', align, copy) with BUILD state (version, byteorder, ...): only plain (non-structured)
    dtypes are accepted."""
    code = node.args[0]
    if not isinstance(code, str) or len(code) > 4:
        raise ValueError(f"refusing dtype {code!r}")
    dt = np.dtype(code)
    order = node.state[1] if isinstance(node.state, tuple) and len(node.state) > 1 else "|"
    if order in ("<", ">"):
        dt = dt.newbyteorder(order)
    if dt.fields is not None:
        raise ValueError("structured dtypes are not supported")
    return dt


def _ndarray_from_state(state: Any) -> np.ndarray:
    """ndarray BUILD state (version, shape, dtype, is_fortran, data): data is raw bytes, or a list of objects for
    dtype=object (each resolved as an inert tree)."""
    _ver, shape, dt, fortran, data = state
    dt = _resolve(dt)
    order = "F" if fortran else "C"
    if dt == np.dtype(object):
        flat = np.empty(len(data), dtype=object)
        for i, v in enumerate(data):
            flat[i] = _resolve(v)
        return flat.reshape(tuple(shape), order=order)
    return np.frombuffer(bytes(data), dtype=dt).reshape(tuple(shape), order=order).copy()


def read_npy_object(path: str) -> Any:
    """``np.save`` of a python object (a 0-d object array, e.g. poselib's Serializable.to_file ``.npy``) read as an
    inert tree -- the non-executing counterpart of ``np.load(path, allow_pickle=True).item()``."""
    with open(path, "rb") as f:
        version = np.lib.format.read_magic(f)
        shape, _fortran, dtype = np.lib.format._read_array_header(f, version)
        if dtype != np.dtype(object):
            f.seek(0)
            return np.lib.format.read_array(f, allow_pickle=False)
        arr = _resolve(_run_vm(io.BytesIO(f.read())))
    return arr.reshape(()).item() if isinstance(arr, np.ndarray) and arr.shape == () else arr


def read_pickle_tree(path: str) -> Any:
    """Read a pickle file into an inert dict/ndarray tree (nothing is executed)."""
    with open(path, "rb") as f:
        data = f.read()
    return _resolve(_run_vm(io.BytesIO(data)))


def load_skeleton_state_arrays(path: str) -> Dict[str, Any]:
    """Extract the arrays of a pickled reference ``SkeletonState``.

    Returns ``node_names``, ``parent_indices`` (int64), ``local_translation``
    (J,3 f32), ``quat`` (J,4 f32, the tree's pre-rotation), ``tensor`` (state
    vector: J*4 rotations then root translation) and ``is_local``.
    Attribute names follow ``poselib/poselib/skeleton/skeleton3d.py:86-95,338-341``.
    """
    tree = read_pickle_tree(path)
    if not (isinstance(tree, dict) and tree.get("__class__", "").endswith("SkeletonState")):
        raise ValueError(f"{path}: not a SkeletonState pickle")
    sk = tree["_skeleton_tree"]
    return {
        "node_names": list(sk["_node_names"]),
        "parent_indices": np.asarray(sk["_parent_indices"], dtype=np.int64),
        "local_translation": np.asarray(sk["_local_translation"], dtype=np.float32),
        "quat": np.asarray(sk["_quat"], dtype=np.float32),
        "tensor": np.asarray(tree["tensor"], dtype=np.float32),
        "is_local": bool(tree["_is_local"]),
    }
