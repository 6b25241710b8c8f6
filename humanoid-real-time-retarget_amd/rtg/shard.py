"""Multi-GPU host logic for the batched retarget path.

Frames are independent, so a global batch shards into contiguous frame ranges,
one per rank, with no data-path collective.  The only collectives are:
  * a broadcast of the packed solver constants (source zero pose: local and
    global translations) from rank 0 at setup;
  * a gather of the per-rank DOF shards to rank 0 after compute;
  * a MAX reduction of the per-rank step time (the bench clock).

Everything here is written against ``torch.distributed`` only, so the same
code runs over RCCL (backend "nccl") on the GPUs and over gloo on CPU tensors
in the world_size-2 tests.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch


def shard_range(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [start, start+count) frame range of ``rank``: the first
    ``total % world`` ranks take one extra frame, so counts differ by <= 1."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} for world {world}")
    if total < 0:
        raise ValueError("total must be >= 0")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, base + (1 if rank < extra else 0)


def pack_solver_consts(zero_local_t: torch.Tensor, zero_global_t: torch.Tensor) -> torch.Tensor:
    """(Js,3) + (Js,3) -> flat float32 blob [Js, local..., global...] (the broadcast payload)."""
    if zero_local_t.shape != zero_global_t.shape or zero_local_t.shape[-1] != 3:
        raise ValueError("zero pose translations must both be (Js, 3)")
    js = torch.tensor([float(zero_local_t.shape[0])], dtype=torch.float32, device=zero_local_t.device)
    return torch.cat([js, zero_local_t.reshape(-1).float(), zero_global_t.reshape(-1).float().to(js.device)])


def unpack_solver_consts(blob: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    js = int(blob[0].item())
    n = js * 3
    if blob.numel() != 1 + 2 * n:
        raise ValueError("malformed solver-constant blob")
    return blob[1:1 + n].reshape(js, 3), blob[1 + n:].reshape(js, 3)


def broadcast_solver_consts(zero_local_t: Optional[torch.Tensor], zero_global_t: Optional[torch.Tensor],
                            max_joints: int, device: torch.device) -> Tuple[torch.Tensor, torch.Tensor]:
    """Rank 0 owns the zero pose; every rank returns identical (local_t, global_t).
    Non-root ranks may pass None.  The blob is sized for ``max_joints`` so the
    receive buffer is known before the payload arrives."""
    import torch.distributed as dist
    cap = 1 + 6 * max_joints
    buf = torch.zeros(cap, dtype=torch.float32, device=device)
    if dist.get_rank() == 0:
        blob = pack_solver_consts(zero_local_t.to(device), zero_global_t.to(device))
        if blob.numel() > cap:
            buf[0] = -1.0          # error marker: every rank raises after the broadcast instead of hanging in it
        else:
            buf[:blob.numel()] = blob
    dist.broadcast(buf, src=0)
    js = int(buf[0].item())
    if js < 0:
        raise ValueError(f"zero pose has more than {max_joints} joints")
    return unpack_solver_consts(buf[:1 + 6 * js])


def pack_setup(parents, local_t, tree_quat, zero_global_t) -> torch.Tensor:
    """Everything a rank needs to build its topology and solver, as one float32 blob:
    [J, parents (J, exact small integers), local_t (J*3), tree_quat (J*4), zero_global_t (J*3)]."""
    p = torch.as_tensor(parents).reshape(-1)
    J = int(p.numel())
    lt, tq, zg = (torch.as_tensor(x).reshape(J, k).float() for x, k in ((local_t, 3), (tree_quat, 4), (zero_global_t, 3)))
    if int(p.min()) < -1 or int(p.max()) >= J:
        raise ValueError("parent indices out of range")
    dev = lt.device
    return torch.cat([torch.tensor([float(J)], device=dev), p.float().to(dev), lt.reshape(-1), tq.to(dev).reshape(-1),
                      zg.to(dev).reshape(-1)])


def unpack_setup(blob: torch.Tensor):
    """-> (parents int32 (J,), local_t (J,3), tree_quat (J,4), zero_global_t (J,3)) as numpy arrays."""
    import numpy as np
    b = blob.detach().cpu()
    J = int(b[0].item())
    if b.numel() != 1 + 11 * J:
        raise ValueError("malformed setup blob")
    o = 1
    parents = b[o:o + J].numpy().astype(np.int32); o += J
    lt = b[o:o + 3 * J].reshape(J, 3).numpy(); o += 3 * J
    tq = b[o:o + 4 * J].reshape(J, 4).numpy(); o += 4 * J
    zg = b[o:o + 3 * J].reshape(J, 3).numpy()
    return parents, lt, tq, zg


def broadcast_setup(setup: Optional[tuple], max_joints: int, device: torch.device):
    """Rank 0 holds (parents, local_t, tree_quat, zero_global_t) of the source skeleton; one broadcast gives every
    rank the same four arrays, so non-root ranks need no local assets (the topology broadcast)."""
    import torch.distributed as dist
    cap = 1 + 11 * max_joints
    buf = torch.zeros(cap, dtype=torch.float32, device=device)
    err = None
    if dist.get_rank() == 0:
        try:
            blob = pack_setup(*setup).to(device)
            if blob.numel() > cap:
                raise ValueError(f"skeleton has more than {max_joints} joints")
            buf[:blob.numel()] = blob
        except ValueError as e:   # still broadcast: the other ranks are already waiting in it
            err = e
            buf[0] = -1.0
    dist.broadcast(buf, src=0)
    J = int(buf[0].item())
    if err is not None:
        raise err
    if J < 0:
        raise ValueError("rank 0 could not pack the setup blob")
    return unpack_setup(buf[:1 + 11 * J])


def max_over_ranks(x: float, device: torch.device) -> float:
    """The bench clock: the slowest rank's elapsed time."""
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_gather_floats(values: Sequence[float], device: torch.device) -> List[List[float]]:
    """Every rank's list of floats (same length on every rank), in rank order, on every rank."""
    import torch.distributed as dist
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    outs = [torch.empty_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(outs, t)
    return [o.cpu().tolist() for o in outs]


def gather_shards(shard: torch.Tensor, counts: Sequence[int], dst: int = 0) -> Optional[torch.Tensor]:
    """Gather ragged contiguous shards (rank r holds ``counts[r]`` leading-dim
    rows) to ``dst`` and concatenate them in rank order; other ranks get None.
    Shards are padded to the largest count because gather needs equal sizes."""
    import torch.distributed as dist
    world, rank = dist.get_world_size(), dist.get_rank()
    if len(counts) != world or shard.shape[0] != counts[rank]:
        raise ValueError("counts must list every rank's shard length")
    m = max(counts) if counts else 0
    if shard.is_cuda and dist.get_backend() == "gloo":   # gloo gathers host tensors only
        shard = shard.cpu()
    padded = shard
    if shard.shape[0] < m:
        padded = torch.cat([shard, shard.new_zeros((m - shard.shape[0],) + tuple(shard.shape[1:]))])
    outs: Optional[List[torch.Tensor]] = [torch.empty_like(padded) for _ in range(world)] if rank == dst else None
    dist.gather(padded.contiguous(), outs, dst=dst)
    if rank != dst:
        return None
    return torch.cat([o[:c] for o, c in zip(outs, counts)])
