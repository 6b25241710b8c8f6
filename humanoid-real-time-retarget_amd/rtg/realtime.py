"""Per-frame teleop path: a resident frame server (FULL_BODY_POS) or one kernel launch over host-mapped pinned
buffers (every kind).

:class:`FrameServer` (rtg_frame_server_launch): one resident workgroup serves frames posted through a sequence
number in pinned memory -- no launch per frame; 26 us median per frame on MI355X (tools/extra_bench.py latency),
bit-identical to the batched solve.  The drop-in retargeters use it for host-input frames (per_frame_runner).

The live loops (sim_full_body_teleop.py:115-119, sim_teleop.py:102) retarget one
frame at a time from host arrays, so a call is launch- and copy-bound, not
compute-bound.  :class:`FrameGraph` packs every input into one pinned staging
buffer that the solver kernel reads directly over the host link, and the kernel
writes local_rot / dof (/ body_rot) straight into one pinned output buffer: a
frame is a host memcpy into the staging buffer, one ``rtg_retarget_f32`` launch
and a wait on a HIP event recorded right after it on a private stream.  The event's
completion signal is written by the command processor after the kernel has ended
(its stores released to the system), so the outputs are read only once they are all
there -- whatever values they hold (round 3 polled the outputs for a sentinel bit
pattern instead, which an input carrying that pattern through a NaN path could mimic).
"""
from __future__ import annotations

import atexit
import ctypes
import time
import weakref
from typing import Sequence

import numpy as np
import torch

from ._lib import FRAME_NAN, RtgError, check, lib
from .runtime import Solver, require_gpu, stream_handle

from .runtime import IN_TAILS as _IN_TAILS

_SERVER_ENDED = 6   # rtg.h RTG_SERVER_ENDED

try:   # the frame's host round trip with tensor arguments and results (rtg/_frame_post.cpp, rtg/build_ext.py)
    from . import _frame_post as _fast_post
except ImportError:   # not built: the ctypes path below does the same call
    _fast_post = None


_F32 = torch.float32


# Device inboxes are pooled for the process, not freed per server: hipFree synchronizes the whole device,
# and dropping one FrameServer while another is resident (its stream busy until it idles out) would stall the caller
# there.  A released inbox goes back to the pool and is handed to the next server; the pool is freed at exit, after
# every server has been closed.
_INBOX_POOL: list = []


def _inbox_take():
    """A device inbox (rtg_server_inbox_alloc) from the pool or a new one, its sequence word 0; None if the device
    has none (no large BAR): the caller keeps a pinned inbox."""
    if _INBOX_POOL:
        p = _INBOX_POOL.pop()
        lib().rtg_frame_server_signal(p, 0)   # a fresh server's ctl[1] is 0: the word must match it (host store only)
        return p
    p = ctypes.c_void_p()
    if lib().rtg_server_inbox_alloc(ctypes.byref(p)) == 0 and p.value:
        return p.value
    return None


def _inbox_give(p) -> None:
    _INBOX_POOL.append(p)


@atexit.register
def _inbox_pool_free() -> None:
    while _INBOX_POOL:
        try:
            lib().rtg_server_inbox_free(_INBOX_POOL.pop())
        except Exception:
            break


def _host_f32_ptr(x, n: int, tail):
    """(address, owner) of n contiguous float32 values on the host: a CPU tensor or array as it is when it already
    is one, else a float32 copy."""
    if type(x) is torch.Tensor and x.is_cpu and x.dtype is _F32 and x.is_contiguous() and x.numel() == n:
        return x.data_ptr(), x   # the teleop loop's case, in five cheap attribute reads
    if isinstance(x, torch.Tensor):
        if x.device.type != "cpu":
            raise ValueError("per-frame inputs are host arrays")
        if x.dtype != torch.float32 or not x.is_contiguous():
            x = x.detach().to(torch.float32).contiguous()
        if x.numel() != n:
            raise ValueError(f"input of {x.numel()} values, expected shape {tail}")
        return x.data_ptr(), x
    a = np.ascontiguousarray(x, dtype=np.float32)
    if a.size != n:
        raise ValueError(f"input of {a.size} values, expected shape {tail}")
    return _addr(a), a


def _addr(a: np.ndarray) -> int:
    return a.__array_interface__["data"][0]   # cheaper than a.ctypes.data


def _marked(dof_row: np.ndarray) -> int:
    """rtg_frame_error code of one frame's host dof row: 0 unless DOF 0 carries the NaN mark (rtg.h RTG_FRAME_NAN)."""
    if dof_row[0] == dof_row[0]:
        return 0
    v = int(dof_row[:1].view(np.uint32)[0])
    return v & 0xF if (v & ~0xF) == FRAME_NAN else 0


class _OutRows:
    """Per-frame output rows carved from blocks of ``n`` frames (one per output; 64 frames, so a view that is pickled drags at most ~100 KB along): a frame's addresses are
    arithmetic and its tensors are views (a numpy index and torch.from_numpy each) -- about 3 us less per frame than
    fresh arrays whose addresses Python has to look up.  A block lives while any frame's tensors do."""

    def __init__(self, shapes, n: int = 64):
        self.shapes, self.n, self.k = shapes, n, n
        self.strides = [4 * int(np.prod(s)) if s else 0 for s in shapes]

    def next(self):
        if self.k == self.n:
            self.blocks = [np.empty((self.n,) + s, np.float32) if s else None for s in self.shapes]
            self.bases = [_addr(b) if b is not None else None for b in self.blocks]
            self.k = 0
        k = self.k
        self.k = k + 1
        return k


class FrameGraph:
    """One frame of a solver kind: (inputs as host arrays) -> (local_rot, dof[, body_rot]) as host tensors."""

    def __init__(self, solver: Solver, want_body_rot: bool = False, timeout_s: float = 2.0):
        dev = require_gpu()
        if dev != solver.device:
            raise ValueError(f"the solver lives on {solver.device}; the current device is {dev}")
        self.solver = solver
        self.tails = _IN_TAILS[solver.kind]
        sizes = [int(np.prod(t)) for t in self.tails]
        self._in_offsets = np.cumsum([0] + sizes)
        self.want_body_rot = bool(want_body_rot)
        n_out = 31 * 4 + 30 + (59 * 4 if want_body_rot else 0)
        # pinned (page-locked, device-mapped) host memory: the kernel reads and writes it directly
        self.h_in = torch.empty(int(self._in_offsets[-1]), dtype=torch.float32).pin_memory()
        self.h_out = torch.empty(n_out, dtype=torch.float32).pin_memory()
        self._h_in_np = self.h_in.numpy()
        base = self.h_in.data_ptr()
        ins = [base + 4 * int(a) for a in self._in_offsets[:-1]] + [None] * (4 - len(sizes))
        out = self.h_out.data_ptr()
        self._args = [solver.handle] + ins + [1, 0, out + 4 * 124, out, out + 4 * 154 if want_body_rot else None]
        # a private stream: the frame never queues behind the caller's batched work, so the time limit measures
        # this launch alone (inputs and outputs are host memory; the solver's constants were made synchronously)
        self.stream = torch.cuda.Stream(dev)
        self.done = torch.cuda.Event()   # no timing: recording and querying it stays cheap
        self.timeout_s = float(timeout_s)
        self.status = 0   # rtg_frame_error code of the last frame

    def _launch(self):
        check(lib().rtg_retarget_f32(*self._args, stream_handle(self.stream)))
        self.done.record(self.stream)

    def _wait(self):
        ev, t0, spins = self.done, None, 0
        while not ev.query():
            spins += 1
            if spins % 256 == 0:
                t0 = t0 or time.perf_counter()
                if time.perf_counter() - t0 > self.timeout_s:
                    raise RtgError(-1, f"rtg_retarget_f32: per-frame launch not done within {self.timeout_s} s")

    def __call__(self, *inputs: Sequence):
        if len(inputs) != len(self.tails):
            raise ValueError(f"expected {len(self.tails)} inputs")
        for x, a, b, t in zip(inputs, self._in_offsets[:-1], self._in_offsets[1:], self.tails):
            arr = x.detach().numpy() if isinstance(x, torch.Tensor) else np.asarray(x)
            if arr.size != b - a:
                raise ValueError(f"input of {arr.size} values, expected shape {t}")
            self._h_in_np[a:b] = arr.reshape(-1)
        self._launch()
        self._wait()
        out = self.h_out.numpy()
        self.status = _marked(out[124:154])   # read by the drop-in retargeters (raise like the reference)
        lr = torch.from_numpy(out[:124].reshape(31, 4).copy())
        dof = torch.from_numpy(out[124:154].copy())
        br = torch.from_numpy(out[154:].reshape(59, 4).copy()) if self.want_body_rot else None
        return lr, dof, br


class FrameServer:
    """FULL_BODY_POS frames served by one resident workgroup (rtg_frame_server_launch): no launch per frame.

    Same call as :class:`FrameGraph` -- (body, left hand, right hand) host arrays -> (local_rot, dof[, body_rot])
    host tensors, bit-identical -- but a frame is a host memcpy into pinned memory plus a sequence-number store; the
    resident kernel sees it, writes the outputs into pinned memory and publishes the number back.  The server ends
    on :meth:`close` (also at exit / garbage collection) or after ``idle_ms`` without a frame; a call after an
    idle exit relaunches it (the pending frame is served by the new launch).  It runs on its own stream, which it
    occupies until it ends: close it before a device-wide synchronize.
    """

    def __init__(self, solver: Solver, want_body_rot: bool = False, idle_ms: int = 200, timeout_s: float = 2.0,
                 device_inbox: bool = True):
        dev = require_gpu()
        if dev != solver.device:
            raise ValueError(f"the solver lives on {solver.device}; the current device is {dev}")
        from ._lib import SERVER_QUIT, SOLVER_FULL_BODY_POS
        if solver.kind != SOLVER_FULL_BODY_POS:
            raise ValueError("FrameServer serves FULL_BODY_POS solvers; use FrameGraph for the other kinds")
        self._quit = np.uint32(SERVER_QUIT)
        self.solver = solver
        self.tails = _IN_TAILS[solver.kind]
        self._in_offsets = np.cumsum([0] + [int(np.prod(t)) for t in self.tails])
        self.want_body_rot = bool(want_body_rot)
        # the inbox (frame + sequence word, rtg.h RTG_SERVER_INBOX_FLOATS): device memory the host stores into through
        # the BAR when the library can map it (4.0 vs 4.8 us per hand-over, tools/bar_probe.hip), else pinned memory
        from ._lib import SERVER_INBOX_FLOATS
        self.h_in = None
        self._inbox = None
        if device_inbox:
            self._inbox = _inbox_take()
        if self._inbox:
            in_ptr = self._inbox
        else:
            self.h_in = torch.zeros(SERVER_INBOX_FLOATS, dtype=torch.float32).pin_memory()
            in_ptr = self.h_in.data_ptr()
        self.h_out = torch.zeros(31 * 4 + 30 + (59 * 4 if want_body_rot else 0), dtype=torch.float32).pin_memory()
        self.h_ctl = torch.zeros(4, dtype=torch.int32).pin_memory()
        self._ctl = self.h_ctl.numpy().view(np.uint32)
        out = self.h_out.data_ptr()
        self._args = [solver.handle, in_ptr, out + 4 * 124, out, out + 4 * 154 if want_body_rot else None,
                      self.h_ctl.data_ptr(), int(idle_ms)]
        self.stream = torch.cuda.Stream(dev)
        self.timeout_s = float(timeout_s)
        self.seq = 0
        self.status = 0   # rtg_frame_error code of the last frame
        self._running = False
        self._sizes = [int(np.prod(t)) for t in self.tails]
        self._rows = _OutRows([(31, 4), (30,), (59, 4) if want_body_rot else None])
        self._post = lib().rtg_frame_server_post
        self._timeout_us = int(self.timeout_s * 1e6)
        self._fast = _fast_post.post if _fast_post is not None else None
        self._post_addr = ctypes.cast(self._post, ctypes.c_void_p).value
        self._ctl_ptr, self._in_ptr = self.h_ctl.data_ptr(), in_ptr
        self._signal = lib().rtg_frame_server_signal
        self._lr_ptr, self._dof_ptr = out, out + 4 * 124
        self._br_ptr = out + 4 * 154 if want_body_rot else None
        ref = weakref.ref(self)   # end the resident kernel at interpreter exit (before HIP tears down)
        self._atexit = lambda: (lambda fs: fs is not None and fs.close())(ref())
        atexit.register(self._atexit)

    def _launch(self):
        self._ctl[2] = 0
        self._ctl[3] = 0
        check(lib().rtg_frame_server_launch(*self._args, stream_handle(self.stream)))
        self._running = True

    def __call__(self, *inputs: Sequence):
        """One frame: the copy in, the post, the wait and the copy out are ONE C call (rtg_frame_server_post).
        Python's share is kept to attribute reads and integer arithmetic (tools/extra_bench.py latency)."""
        if len(inputs) != 3:
            raise ValueError("expected 3 inputs")
        b, lh, rh = inputs
        if self._fast is not None and type(b) is torch.Tensor and type(lh) is torch.Tensor and type(rh) is torch.Tensor:
            if not self._running or (self._ctl[2] and self.stream.query()):
                self._launch()
            self.seq = self.seq + 1 if self.seq + 1 < int(self._quit) else 1
            args = (self._post_addr, self._ctl_ptr, self.seq, self._in_ptr, b, lh, rh, self._dof_ptr, self._lr_ptr,
                    self._br_ptr or 0, self._timeout_us)
            rc, code, lr, dof, br = self._fast(*args)
            while rc == _SERVER_ENDED:   # idled out before it took the frame: relaunch (the frame is still posted)
                self.stream.synchronize()
                self._launch()
                rc, code, lr, dof, br = self._fast(*args)
            if rc != _fast_post.NOT_HOST_F32:   # else: inputs to convert, the ctypes path below
                check(rc)
                self.status = code
                return lr, dof, br
        sz, tl = self._sizes, self.tails
        p0, x0 = _host_f32_ptr(inputs[0], sz[0], tl[0])
        p1, x1 = _host_f32_ptr(inputs[1], sz[1], tl[1])
        p2, x2 = _host_f32_ptr(inputs[2], sz[2], tl[2])
        R = self._rows
        k = R.next()
        (b_lr, b_dof, b_br), (s_lr, s_dof, s_br) = R.bases, R.strides
        if not self._running or (self._ctl[2] and self.stream.query()):
            self._launch()
        self.seq = self.seq + 1 if self.seq + 1 < int(self._quit) else 1
        args = (self._ctl_ptr, self.seq, self._in_ptr, p0, p1, p2, self._dof_ptr, self._lr_ptr, self._br_ptr,
                b_dof + k * s_dof, b_lr + k * s_lr, b_br + k * s_br if b_br is not None else None, self._timeout_us)
        rc = self._post(*args)
        while rc == _SERVER_ENDED:   # it idled out before it took the frame: relaunch (the frame is still posted)
            self.stream.synchronize()
            self._launch()
            rc = self._post(*args)
        check(rc)
        lr, dof, br = R.blocks
        dof = dof[k]
        self.status = _marked(dof)
        return torch.from_numpy(lr[k]), torch.from_numpy(dof), (torch.from_numpy(br[k]) if br is not None else None)

    def close(self):
        if self._running:
            self._signal(self._in_ptr, int(self._quit))
            self.stream.synchronize()
            self._running = False
            self._ctl[1] = self.seq   # a relaunch starts from the last posted frame: word == ctl[1]
            self._signal(self._in_ptr, self.seq)
        fn = getattr(self, "_atexit", None)
        if fn is not None:
            atexit.unregister(fn)
            self._atexit = None

    def _release(self):
        """The device inbox back to the process pool -- no hipFree here (a device-wide synchronize).  Only once the
        server has ended: a resident kernel still polls its inbox."""
        if getattr(self, "_running", False):
            return
        inbox, self._inbox = getattr(self, "_inbox", None), None
        if inbox:
            _inbox_give(inbox)

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            try:
                self.close()
            finally:
                self._release()
        except Exception:
            pass


def per_frame_runner(solver: Solver, want_body_rot: bool = False, server: bool = False, idle_ms: int = 200):
    """The per-frame call the drop-in retargeters use for host inputs: :class:`FrameGraph` (one launch per frame,
    nothing resident), or with ``server`` the resident :class:`FrameServer` (FULL_BODY_POS only)."""
    from ._lib import SOLVER_FULL_BODY_POS
    if server and solver.kind == SOLVER_FULL_BODY_POS:
        return FrameServer(solver, want_body_rot, idle_ms=idle_ms)
    return FrameGraph(solver, want_body_rot)
