"""Per-frame teleop path: one kernel launch over host-mapped pinned buffers.

The live loops (sim_full_body_teleop.py:115-119, sim_teleop.py:102) retarget one
frame at a time from host arrays, so a call is launch- and copy-bound, not
compute-bound.  :class:`FrameGraph` packs every input into one pinned staging
buffer that the solver kernel reads directly over the host link, and the kernel
writes local_rot / dof (/ body_rot) straight into one pinned output buffer: a
frame is a host memcpy into the staging buffer, one ``rtg_retarget_f32`` launch
(no copy nodes, no graph), and a spin on the output buffer itself.

Completion is seen in the outputs: before the launch every output word is set
to a signalling-NaN payload (0x7FBADBAD) that the kernel never stores -- every
value it writes is arithmetic (quieted NaNs set bit 22) or a constant -- so the
call returns once no word holds it.  A stream query every few hundred spins
catches a launch that finished without writing (an error) and a time limit
ends a hung one.  Measured on MI355X (tools/latency_phases.py): 44 us median
per frame against 61 us for the earlier captured graph with H2D / D2H copy
nodes, bit-identical outputs.
"""
from __future__ import annotations

import time
from typing import Sequence

import numpy as np
import torch

from ._lib import RtgError, check, lib
from .runtime import Solver, require_gpu, stream_handle

from .runtime import IN_TAILS as _IN_TAILS

SENTINEL = np.uint32(0x7FBADBAD)


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
        self._out_u32 = self.h_out.numpy().view(np.uint32)
        self._dof_u32 = self._out_u32[124:154]
        base = self.h_in.data_ptr()
        ins = [base + 4 * int(a) for a in self._in_offsets[:-1]] + [None] * (4 - len(sizes))
        out = self.h_out.data_ptr()
        self._args = [solver.handle] + ins + [1, 0, out + 4 * 124, out, out + 4 * 154 if want_body_rot else None]
        self.stream = torch.cuda.current_stream(dev)
        self.timeout_s = float(timeout_s)

    def _launch(self):
        check(lib().rtg_retarget_f32(*self._args, stream_handle(self.stream)))

    def _wait(self):
        u, d = self._out_u32, self._dof_u32
        spins, t0 = 0, None
        while True:
            if not (d == SENTINEL).any() and not (u == SENTINEL).any():   # the 30 DOF words first: a cheap gate
                return
            spins += 1
            if spins % 256 == 0:
                if self.stream.query() and (u == SENTINEL).any():
                    raise RtgError(-1, "rtg_retarget_f32: the per-frame launch completed without writing its outputs")
                t0 = t0 or time.perf_counter()
                if time.perf_counter() - t0 > self.timeout_s:
                    raise RtgError(-1, f"rtg_retarget_f32: per-frame outputs not written within {self.timeout_s} s")

    def __call__(self, *inputs: Sequence):
        if len(inputs) != len(self.tails):
            raise ValueError(f"expected {len(self.tails)} inputs")
        for x, a, b, t in zip(inputs, self._in_offsets[:-1], self._in_offsets[1:], self.tails):
            arr = x.detach().numpy() if isinstance(x, torch.Tensor) else np.asarray(x)
            if arr.size != b - a:
                raise ValueError(f"input of {arr.size} values, expected shape {t}")
            self._h_in_np[a:b] = arr.reshape(-1)
        self._out_u32[...] = SENTINEL
        self._launch()
        self._wait()
        out = self.h_out.numpy()
        lr = torch.from_numpy(out[:124].reshape(31, 4).copy())
        dof = torch.from_numpy(out[124:154].copy())
        br = torch.from_numpy(out[154:].reshape(59, 4).copy()) if self.want_body_rot else None
        return lr, dof, br
