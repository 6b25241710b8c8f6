"""world_size-2 gloo tests of the multi-GPU host logic (rtg/shard.py, bench.py's N>1 path) on CPU."""
from __future__ import annotations

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG  # noqa: F401  (puts the package on sys.path)
from rtg import shard


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world)))
    except Exception as e:  # noqa: BLE001
        q.put((rank, e))
    finally:
        dist.destroy_process_group()


def _run(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r, v in res.items():
        if isinstance(v, Exception):
            raise v
    return res


def test_shard_range_partitions():
    for total in (0, 1, 7, 262144, 2 * 1024 * 1024 + 3):
        for world in (1, 2, 3, 8):
            spans = [shard.shard_range(total, world, r) for r in range(world)]
            assert spans[0][0] == 0 and sum(c for _, c in spans) == total
            for (s0, c0), (s1, _) in zip(spans, spans[1:]):
                assert s0 + c0 == s1
            assert max(c for _, c in spans) - min(c for _, c in spans) <= 1
    with pytest.raises(ValueError):
        shard.shard_range(10, 2, 2)


def test_pack_roundtrip():
    zl, zg = torch.randn(59, 3), torch.randn(59, 3)
    a, b = shard.unpack_solver_consts(shard.pack_solver_consts(zl, zg))
    assert torch.equal(a, zl) and torch.equal(b, zg)
    with pytest.raises(ValueError):
        shard.pack_solver_consts(zl, zg[:5])


def _bcast(rank, world):
    from rtg import assets
    zl = torch.from_numpy(assets.local_translation("vtrdyn_full")) if rank == 0 else None
    zg = torch.arange(177, dtype=torch.float32).reshape(59, 3) if rank == 0 else None
    a, b = shard.broadcast_solver_consts(zl, zg, max_joints=64, device=torch.device("cpu"))
    return a.numpy(), b.numpy()


def test_broadcast_solver_consts_world2():
    from rtg import assets
    res = _run(_bcast)
    for r in (0, 1):
        np.testing.assert_array_equal(res[r][0], assets.local_translation("vtrdyn_full"))
        np.testing.assert_array_equal(res[r][1], np.arange(177, dtype=np.float32).reshape(59, 3))


def _gather_ragged(rank, world):
    total = 11
    start, count = shard.shard_range(total, world, rank)
    full = torch.arange(total * 30, dtype=torch.float32).reshape(total, 30)
    mine = full[start:start + count].clone()
    counts = [shard.shard_range(total, world, r)[1] for r in range(world)]
    out = shard.gather_shards(mine, counts)
    t = shard.max_over_ranks(float(rank + 1), torch.device("cpu"))
    return (None if out is None else out.numpy()), t


def test_gather_and_max_world2():
    res = _run(_gather_ragged)
    np.testing.assert_array_equal(res[0][0], np.arange(330, dtype=np.float32).reshape(11, 30))
    assert res[1][0] is None
    assert res[0][1] == res[1][1] == 2.0


def _sharded_solve(rank, world):
    """bench.py's data flow at world 2 with the oracle standing in for the device solver:
    per-rank seeded shards, broadcast constants, local solve, gather -> identical to a 1-rank solve."""
    import oracle as orc
    from rtg import synth
    zp = np.load(os.path.join(os.path.dirname(__file__), "golden", "zero_pose.npz"))
    zl_t = torch.from_numpy(zp["vtrdyn_full_local_t"]) if rank == 0 else None
    zg_t = torch.from_numpy(zp["vtrdyn_full_global_t"]) if rank == 0 else None
    zl, zg = shard.broadcast_solver_consts(zl_t, zg_t, 64, torch.device("cpu"))
    total = 37
    body, lh, rh = synth.synth_full_body_inputs(total, seed=99)
    start, count = shard.shard_range(total, world, rank)
    sl = slice(start, start + count)
    dof, _, _ = orc.full_body_pos(zl.numpy(), zg.numpy(), body[sl], lh[sl], rh[sl], True, want_rot=False)
    counts = [shard.shard_range(total, world, r)[1] for r in range(world)]
    out = shard.gather_shards(torch.from_numpy(np.ascontiguousarray(dof)), counts)
    return None if out is None else out.numpy()


def test_sharded_solve_matches_single_rank():
    import oracle as orc
    from rtg import synth
    res = _run(_sharded_solve)
    zp = np.load(os.path.join(os.path.dirname(__file__), "golden", "zero_pose.npz"))
    body, lh, rh = synth.synth_full_body_inputs(37, seed=99)
    ref, _, _ = orc.full_body_pos(zp["vtrdyn_full_local_t"], zp["vtrdyn_full_global_t"], body, lh, rh, True,
                                  want_rot=False)
    np.testing.assert_array_equal(res[0], ref)


from bench_host_backend import HostBackend  # noqa: E402  (bench.DeviceBackend's interface, oracle inside)


def _bench_flow(rank, world):
    import bench
    from rtg import assets
    if rank != 0:   # non-root ranks must get the skeleton from the broadcast, not from local assets
        def _no_assets(*a, **k):
            raise AssertionError("rank > 0 read a local asset")
        for name in ("parents", "local_translation", "tree_quat"):
            setattr(assets, name, _no_assets)
    res = bench.rank_flow(world, rank, HostBackend(), B=23, steps=3, warmup=1, ring=2)
    g = res.get("gathered")
    return {"gathered": None if g is None else g.numpy(), "wall": res["wall"], "frames": res["frames"],
            "zg": np.asarray(res["zg"]), "parents": np.asarray(res["parents"])}


def test_bench_rank_flow_world2():
    """bench.py's N>1 flow (rank_flow) at world 2 over gloo with a host stand-in for the device launch: the setup
    broadcast carries the topology (rank 1 reads no assets), each rank solves its own seeded shard, the clock is
    the max over ranks, and rank 0's gather equals solving both shards on one rank."""
    import oracle as orc
    from rtg import assets, synth
    res = _run(_bench_flow)
    assert res[0]["wall"] == res[1]["wall"] and res[0]["frames"] == res[1]["frames"] == 2 * 23 * 3
    np.testing.assert_array_equal(res[0]["parents"], assets.parents("vtrdyn_full"))
    np.testing.assert_array_equal(res[1]["parents"], assets.parents("vtrdyn_full"))
    np.testing.assert_array_equal(res[0]["zg"], res[1]["zg"])
    np.testing.assert_array_equal(res[0]["zg"], np.load(os.path.join(os.path.dirname(__file__), "golden",
                                                                     "zero_pose.npz"))["vtrdyn_full_global_t"])
    assert res[1]["gathered"] is None
    zg, zl = res[0]["zg"], assets.local_translation("vtrdyn_full")
    want = []
    for rank in (0, 1):   # the last timed step used ring set (3 - 1) % 2 = 0: frame offset 0
        b, l, r = synth.synth_full_body_inputs(23, seed=(1234 + rank) * 1000)
        want.append(orc.full_body_pos(zl, zg, b, l, r, True, want_rot=False)[0])
    np.testing.assert_array_equal(res[0]["gathered"], np.concatenate(want))


def test_setup_blob_roundtrip():
    from rtg import assets
    p, lt, tq = assets.parents("vtrdyn_full"), assets.local_translation("vtrdyn_full"), assets.tree_quat("vtrdyn_full")
    zg = np.arange(177, dtype=np.float32).reshape(59, 3)
    a, b, c, d = shard.unpack_setup(shard.pack_setup(p, lt, tq, zg))
    np.testing.assert_array_equal(a, p)
    np.testing.assert_array_equal(b, lt)
    np.testing.assert_array_equal(c, tq)
    np.testing.assert_array_equal(d, zg)
    with pytest.raises(ValueError):
        shard.pack_setup(np.int32([-1, 0, 5]), lt[:3], tq[:3], zg[:3])


def _bench_cmd(*extra, env_extra=None):
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(RTG_BENCH_BACKEND="bench_host_backend:HostBackend",
               PYTHONPATH=os.pathsep.join([os.path.dirname(os.path.abspath(__file__)), repo, env.get("PYTHONPATH", "")]))
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(repo, "bench.py"), *extra], env=env, capture_output=True,
                          text=True, timeout=300)


def test_bench_gpus_flag_spawns_ranks_world2():
    """`python bench.py --gpus 2` with no launcher environment starts two rank processes itself (the driver's
    N-GPU invocation): rank 0 prints n_gpus 2, both ranks report their own golden check, the clock is the max over
    ranks, and the gathered DOFs equal solving both seeded shards on one rank."""
    import hashlib
    import json
    import oracle as orc
    from rtg import assets, synth
    r = _bench_cmd("--gpus", "2", "--steps", "3", "--warmup", "1", "--batch", "23", "--ring", "2")
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["backend"] == "HostBackend"
    ranks = line["golden_per_rank"]
    assert [g["rank"] for g in ranks] == [0, 1]
    for g in ranks:
        assert g["frames"] == 512 and g["max_abs_err"] <= 2.2e-5
    zp = np.load(os.path.join(os.path.dirname(__file__), "golden", "zero_pose.npz"))
    want = []
    for rank in (0, 1):   # the last timed step used ring set (3 - 1) % 2 = 0: frame offset 0
        b, l, rr = synth.synth_full_body_inputs(23, seed=(1234 + rank) * 1000)
        want.append(orc.full_body_pos(assets.local_translation("vtrdyn_full"), zp["vtrdyn_full_global_t"], b, l, rr,
                                      True, want_rot=False)[0])
    assert line["gathered_sha1"] == hashlib.sha1(np.ascontiguousarray(np.concatenate(want)).tobytes()).hexdigest()
    # the line proves its N: one device identity per rank, all distinct, and the collective backend used
    assert [d["rank"] for d in line["devices"]] == [0, 1]
    assert len({d["pci"] for d in line["devices"]}) == 2
    assert line["comm"]["backend"] == "gloo" and line["comm"]["world"] == 2


def test_bench_refuses_two_ranks_on_one_device():
    """Two ranks reporting the same device identity: every rank raises before the timed region (none hangs in a
    collective) and no line is printed."""
    r = _bench_cmd("--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "8", "--ring", "2",
                   env_extra={"RTG_TEST_SAME_DEVICE": "1"})
    assert r.returncode != 0
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert "2 ranks on 1 distinct devices" in r.stderr


def test_bench_gpus_flag_must_match_launcher_world():
    r = _bench_cmd("--gpus", "1", "--steps", "1", env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "disagrees with WORLD_SIZE" in r.stderr


def _bcast_too_big(rank, world):
    J = 9
    setup = (np.arange(-1, J - 1, dtype=np.int32), np.zeros((J, 3), np.float32), np.tile(np.float32([0, 0, 0, 1]), (J, 1)),
             np.zeros((J, 3), np.float32)) if rank == 0 else None
    try:
        shard.broadcast_setup(setup, max_joints=4, device=torch.device("cpu"))
    except ValueError as e:
        return str(e)
    return "no error"


def test_broadcast_setup_error_reaches_every_rank():
    """A skeleton larger than the broadcast buffer raises on EVERY rank (rank 0 still joins the broadcast with an
    error marker) instead of leaving the other ranks blocked in it."""
    res = _run(_bcast_too_big)
    assert "more than 4 joints" in res[0]
    assert "could not pack" in res[1]
