"""bench.DeviceBackend's interface with the oracle standing in for the device launch (gloo, CPU tensors).

Test infrastructure only: it lets the world-size-2 tests run bench.py's own N>1 flow -- rank_flow, and the
``--gpus N`` launcher through ``RTG_BENCH_BACKEND=bench_host_backend:HostBackend`` -- without a GPU.
"""
from __future__ import annotations

import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))


class HostBackend:
    DIST_BACKEND = "gloo"

    @staticmethod
    def bind_device(local):
        pass

    @staticmethod
    def pg_kwargs(local):
        return {}

    def __init__(self, local=0):
        self.comm_device = torch.device("cpu")

    def zero_global(self, parents, lt, tq):
        import oracle as orc
        J = len(parents)
        _, gp = orc.state_fk(parents, tq, lt, np.tile(np.float32([0, 0, 0, 1]), (1, J, 1)), np.zeros((1, 3), np.float32))
        return gp[0]

    def build(self, parents, lt, tq, zg):
        return ("topo", np.asarray(parents)), ("solver", np.asarray(lt, np.float32), np.asarray(zg, np.float32))

    def synth(self, topo, B, seed, offset):
        from rtg import synth
        return tuple(torch.from_numpy(a) for a in synth.synth_full_body_inputs(B, seed=seed * 1000 + offset))

    def new_dof(self, B):
        return torch.empty((B, 30), dtype=torch.float32)

    def solve(self, solver, b, l, r, d):
        import oracle as orc
        dof, _, _ = orc.full_body_pos(solver[1], solver[2], b.numpy(), l.numpy(), r.numpy(), True, want_rot=False)
        d.copy_(torch.from_numpy(dof))

    def golden_check(self, solver):
        import bench
        import oracle as orc
        g = np.load(os.path.join(HERE, "golden", "full_body_pos_precise.npz"))
        dof, _, _ = orc.full_body_pos(solver[1], solver[2], g["body"], g["lh"], g["rh"], True, want_rot=False)
        return bench.golden_errors(dof, g["dof"])

    def sync(self):
        pass

    def identity(self):
        """A stand-in device identity: this rank's process (RTG_TEST_SAME_DEVICE=1 makes every rank report the
        same one, to test that rank_flow refuses it)."""
        if os.environ.get("RTG_TEST_SAME_DEVICE") == "1":
            return {"name": "host", "pci": "host-0", "uuid": None}
        return {"name": "host", "pci": f"host-pid-{os.getpid()}", "uuid": None}

    def start(self):
        pass

    def stop(self):
        pass

    def elapsed_ms(self):
        return 1.0
