"""bench.DeviceBackend with every rank on cuda:0 and gloo for the collectives: a one-GPU rehearsal of bench.py's
N>1 device path (two streams per rank, the clock settle, the single-launch kernel time, the max over ranks, the
golden check per rank and the DOF gather).  RCCL refuses two ranks on one device, so this is the only way the
N-rank device flow runs on the one-GPU box; the driver's N-GPU run uses DeviceBackend itself (RCCL, one GPU per
rank).  Test infrastructure only (tests/test_gpu_edge.py)."""
from __future__ import annotations

import torch

from bench import DeviceBackend


class SharedGpuGlooBackend(DeviceBackend):
    DIST_BACKEND = "gloo"
    SHARES_DEVICE = True   # every rank on cuda:0 on purpose: rank_flow's distinct-device check is waived

    @staticmethod
    def bind_device(local):
        torch.cuda.set_device(0)

    @staticmethod
    def pg_kwargs(local):
        return {}

    def __init__(self, local, layout="soa"):
        super().__init__(0, layout)
        self.comm_device = torch.device("cpu")
