"""Per-frame teleop path as one replayable HIP graph.

The live loops (sim_full_body_teleop.py:115-119, sim_teleop.py:102) retarget one
frame at a time from host arrays, so a call is launch- and copy-bound, not
compute-bound.  :class:`FrameGraph` packs every input into one pinned staging
buffer, and captures -- once -- one H2D copy, the solver launch
(``rtg_retarget_f32``) and one D2H copy of all outputs into a HIP graph (via
``torch.cuda.graph``).  A frame is then: host memcpy into the staging buffer,
``graph.replay()``, one stream synchronise.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch

from ._lib import check, lib
from .runtime import Solver, ptr, require_gpu, stream_handle

from .runtime import IN_TAILS as _IN_TAILS


class FrameGraph:
    """One frame of a solver kind, captured as a graph: (inputs as host arrays) -> (local_rot, dof[, body_rot])."""

    def __init__(self, solver: Solver, want_body_rot: bool = False):
        dev = require_gpu()
        self.solver = solver
        self.tails = _IN_TAILS[solver.kind]
        sizes = [int(np.prod(t)) for t in self.tails]
        self._in_offsets = np.cumsum([0] + sizes)
        n_in = int(self._in_offsets[-1])
        self.want_body_rot = bool(want_body_rot)
        n_out = 31 * 4 + 30 + (59 * 4 if want_body_rot else 0)
        self.h_in = torch.empty(n_in, dtype=torch.float32).pin_memory()
        self.h_out = torch.empty(n_out, dtype=torch.float32).pin_memory()
        self.d_in = torch.zeros(n_in, dtype=torch.float32, device=dev)
        self.d_out = torch.zeros(n_out, dtype=torch.float32, device=dev)
        self._h_in_np = self.h_in.numpy()
        self._h_out_np = self.h_out.numpy()
        self._ins = [self.d_in[a:b] for a, b in zip(self._in_offsets[:-1], self._in_offsets[1:])]
        self._lr, self._dof = self.d_out[:124], self.d_out[124:154]
        self._br = self.d_out[154:] if want_body_rot else None
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):   # warm-up outside the capture
            for _ in range(2):
                self._step()
        torch.cuda.current_stream().wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, stream=s):
            self._step()
        torch.cuda.synchronize()

    def _step(self):
        self.d_in.copy_(self.h_in, non_blocking=True)
        ins: List = [ptr(t) for t in self._ins] + [None] * (4 - len(self._ins))
        check(lib().rtg_retarget_f32(self.solver.handle, ins[0], ins[1], ins[2], ins[3], 1, 0, ptr(self._dof),
                                     ptr(self._lr), ptr(self._br), stream_handle()))
        self.h_out.copy_(self.d_out, non_blocking=True)

    def __call__(self, *inputs: Sequence):
        if len(inputs) != len(self.tails):
            raise ValueError(f"expected {len(self.tails)} inputs")
        for x, a, b, t in zip(inputs, self._in_offsets[:-1], self._in_offsets[1:], self.tails):
            arr = x.detach().numpy() if isinstance(x, torch.Tensor) else np.asarray(x)
            if arr.size != b - a:
                raise ValueError(f"input of {arr.size} values, expected shape {t}")
            self._h_in_np[a:b] = arr.reshape(-1)
        self.graph.replay()
        torch.cuda.current_stream().synchronize()
        out = self._h_out_np
        lr = torch.from_numpy(out[:124].reshape(31, 4).copy())
        dof = torch.from_numpy(out[124:154].copy())
        br = torch.from_numpy(out[154:].reshape(59, 4).copy()) if self.want_body_rot else None
        return lr, dof, br
