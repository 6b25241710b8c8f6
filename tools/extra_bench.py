"""Secondary measurements (not the driver's bench line):

  latency  -- batch-1 / small-batch retarget latency (teleop path, SURVEY §7 "Latency path"):
              kernel-only (HIP events) and end-to-end host->device->host wall time
  fk       -- FK throughput: Hu (B=262144) and the mixed 4-topology config (4 x 65536, one launch)
  solvers  -- throughput of all four solver kinds at B=262144
"""
from __future__ import annotations

import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "humanoid-real-time-retarget_amd"))

from rtg import _lib, assets, ops, synth  # noqa: E402
from rtg.runtime import Solver, Topology  # noqa: E402

G = os.path.join(REPO, "tests", "golden")


def topo(name):
    return Topology(assets.parents(name), assets.local_translation(name), assets.tree_quat(name))


def time_events(fn, reps=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def latency():
    zp = np.load(os.path.join(G, "zero_pose.npz"))
    g = np.load(os.path.join(G, "full_body_pos_precise.npz"))
    S = Solver(_lib.SOLVER_FULL_BODY_POS, zp["vtrdyn_full_local_t"], zp["vtrdyn_full_global_t"],
               assets.parents("vtrdyn_full"), True)
    out = {}
    for B in (1, 16, 256, 4096):
        idx = np.arange(B) % len(g["body"])
        hb, hl, hr = (np.ascontiguousarray(g[k][idx]) for k in ("body", "lh", "rh"))
        db, dl, dr = (torch.from_numpy(a).cuda() for a in (hb, hl, hr))
        dof = torch.empty((B, 30), device="cuda")
        k_ms = time_events(lambda: S.retarget([db, dl, dr], out_dof=dof))
        pb, pl, pr = (torch.from_numpy(a).pin_memory() for a in (hb, hl, hr))
        hdof = torch.empty((B, 30)).pin_memory()

        def e2e():
            db.copy_(pb, non_blocking=True); dl.copy_(pl, non_blocking=True); dr.copy_(pr, non_blocking=True)
            S.retarget([db, dl, dr], out_dof=dof)
            hdof.copy_(dof, non_blocking=True)
            torch.cuda.current_stream().synchronize()
        for _ in range(10):
            e2e()
        ts = []
        for _ in range(200):
            t0 = time.perf_counter()
            e2e()
            ts.append(time.perf_counter() - t0)
        out[str(B)] = {"kernel_us": k_ms * 1e3, "e2e_median_us": float(np.median(ts) * 1e6),
                       "e2e_p99_us": float(np.quantile(ts, 0.99) * 1e6)}
    # the drop-in per-frame call of the teleop loop (host tensors in/out; captured HIP graph, rtg.realtime)
    from rtg.realtime import FrameGraph
    sys.path.insert(0, os.path.join(REPO, "humanoid-real-time-retarget_amd"))
    from retarget.retarget_solver import VtrdynFullBodyPosRetargeter
    from robot_kinematics_model import RobotZeroPose
    hu = VtrdynFullBodyPosRetargeter(RobotZeroPose.from_asset("vtrdyn_full"), RobotZeroPose.from_asset("hu_v5"),
                                     precise_gripper=True)
    fb, fl, fr = (torch.from_numpy(np.ascontiguousarray(g[k][0])) for k in ("body", "lh", "rh"))
    from rtg.realtime import FrameServer
    fg = FrameGraph(S, want_body_rot=False)
    fsrv = FrameServer(S, want_body_rot=False)
    fsrv_br = FrameServer(S, want_body_rot=True)
    fsrv_pin = FrameServer(S, want_body_rot=False, device_inbox=False)   # round 4's inbox: pinned host memory
    for name, fn in (("dropin_retarget_per_frame", lambda: hu.retarget(fb, fl, fr)),
                     ("frame_server_dof_local_rot_body_rot", lambda: fsrv_br(fb, fl, fr)),
                     ("dropin_batch_of_one_no_graph",
                      lambda: hu.retarget_batch(fb[None], fl[None], fr[None], want_body_rot=True)),
                     ("frame_graph_dof_local_rot", lambda: fg(fb, fl, fr)),
                     ("frame_server_dof_local_rot", lambda: fsrv(fb, fl, fr)),
                     ("frame_server_dof_local_rot_pinned_inbox", lambda: fsrv_pin(fb, fl, fr)),
                     ("frame_server_dof_local_rot_again", lambda: fsrv(fb, fl, fr))):
        for _ in range(20):
            fn()
        ts = []
        for _ in range(500):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        out[name] = {"median_us": float(np.median(ts) * 1e6), "p99_us": float(np.quantile(ts, 0.99) * 1e6)}
    a, b = fg(fb, fl, fr), fsrv(fb, fl, fr)
    out["frame_server_bits_equal_frame_graph"] = bool(torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]))
    out["frame_server_inbox_in_device_memory"] = fsrv._inbox is not None
    fsrv.close()
    fsrv_br.close()
    fsrv_pin.close()
    hu.close()
    return out


def teleop_gaps():
    """The teleop loop's per-frame call with the loop's own work between frames: the reference's
    sim_full_body_teleop.py:91-126 follows every retarget with a MuJoCo step, a viewer render and a recorder call,
    so frames arrive every few to tens of ms.  For each gap (a sleep between calls, excluded from the timing) the
    drop-in retarget() is timed with the resident frame server at several idle_ms (the server ends after idle_ms
    without a frame and is relaunched by the next one) and with the one-launch FrameGraph (frame_server=False)."""
    sys.path.insert(0, os.path.join(REPO, "humanoid-real-time-retarget_amd"))
    from retarget.retarget_solver import VtrdynFullBodyPosRetargeter
    from robot_kinematics_model import RobotZeroPose
    g = np.load(os.path.join(G, "full_body_pos_precise.npz"))
    fb, fl, fr = (torch.from_numpy(np.ascontiguousarray(g[k][0])) for k in ("body", "lh", "rh"))
    configs = [("frame_server_idle5", True, 5), ("frame_server_idle50", True, 50), ("frame_server_idle200", True, 200),
               ("frame_graph", False, 5)]
    out = {}
    n = int(os.environ.get("RTG_GAP_FRAMES", "60"))
    for gap_ms in (0, 2, 5, 10, 20, 33):
        row = {}
        for name, server, idle in configs:
            hu = VtrdynFullBodyPosRetargeter(RobotZeroPose.from_asset("vtrdyn_full"), RobotZeroPose.from_asset("hu_v5"),
                                             precise_gripper=True, frame_server=server, idle_ms=idle)
            for _ in range(5):
                hu.retarget(fb, fl, fr)
            ts = []
            for _ in range(n):
                if gap_ms:
                    time.sleep(gap_ms * 1e-3)
                t0 = time.perf_counter()
                hu.retarget(fb, fl, fr)
                ts.append(time.perf_counter() - t0)
            hu.close()
            row[name] = {"median_us": round(float(np.median(ts) * 1e6), 1),
                         "p90_us": round(float(np.quantile(ts, 0.9) * 1e6), 1)}
        out[f"gap_{gap_ms}ms"] = row
        print(gap_ms, row, flush=True)
    return out


def fk():
    """Kinematics kernels through the C ABI with every output preallocated and the ctypes arguments built once: a
    Python-level call (ops.*) allocates its outputs and costs 30-130 us of host time, above some of these kernels'
    own time, so back-to-back ops.* calls timed the host (round 5's 'k_dof_fk 128 us' was that)."""
    from rtg._lib import check, lib
    from rtg.runtime import DofModel, ptr, stream_handle
    import importlib
    res = {}
    B = 262144
    sh = stream_handle()
    T = topo("hu_v5")
    lr = torch.from_numpy(synth.random_local_quats(B, 31, 5)).cuda()
    rt = torch.zeros((B, 3), device="cuda")
    gr = torch.empty((B, 31, 4), device="cuda")
    gp = torch.empty((B, 31, 3), device="cuda")
    fk_args = (T.handle, ptr(lr), ptr(rt), B, ptr(gr), ptr(gp), sh)
    f = lib().rtg_fk_f32
    ms = time_events(lambda: f(*fk_args))
    check(f(*fk_args))
    res["hu_fk_262144"] = {"ms": ms, "frames_per_s": B / (ms * 1e-3),
                           "GBs_algorithmic": 1376 * B / (ms * 1e-3) / 1e9}
    lo = torch.empty((B, 31, 4), device="cuda")
    inv_args = (T.handle, ptr(gr), B, ptr(lo), sh)
    f = lib().rtg_local_rotation_f32
    ms = time_events(lambda: f(*inv_args))
    check(f(*inv_args))
    res["hu_inverse_fk_262144"] = {"ms": ms, "frames_per_s": B / (ms * 1e-3),
                                   "GBs_algorithmic": 31 * 32 * B / (ms * 1e-3) / 1e9}
    # HuForwardModel: joint angles -> FK (33-link Hu, clip on): (J-1)*4 + 16 + 12 in, J*28 out per frame
    hu = importlib.import_module("retarget.robot_config.Hu")
    Th = topo("hu")
    M = DofModel(Th, hu.Hu_DOF_AXIS, hu.Hu_DOF_LOWER.numpy(), hu.Hu_DOF_UPPER.numpy())
    dof = (torch.rand((B, 32), device="cuda") - 0.5) * 4
    rr = torch.nn.functional.normalize(torch.randn((B, 4), device="cuda"), dim=-1)
    dgr = torch.empty((B, 33, 4), device="cuda")
    dgp = torch.empty((B, 33, 3), device="cuda")
    dof_args = (M.handle, ptr(dof), ptr(rr), ptr(rt), B, 1, ptr(dgr), ptr(dgp), sh)
    f = lib().rtg_dof_fk_f32
    ms = time_events(lambda: f(*dof_args))
    check(f(*dof_args))
    res["hu_dof_fk_262144"] = {"ms": ms, "frames_per_s": B / (ms * 1e-3),
                               "GBs_algorithmic": (32 * 4 + 28 + 33 * 28) * B / (ms * 1e-3) / 1e9}
    segs = []
    nbytes = 0
    for i, n in enumerate(["hu_v5", "vtrdyn", "vtrdyn_full", "noitom"]):
        t = topo(n)
        J = t.num_joints
        segs.append((t, torch.from_numpy(synth.random_local_quats(65536, J, 10 + i)).cuda(),
                     torch.zeros((65536, 3), device="cuda")))
        nbytes += 65536 * (J * 16 + 12 + J * 28)
    fsegs, keep, outs = ops._fk_segments(segs)
    f = lib().rtg_fk_multi_f32
    ms = time_events(lambda: f(fsegs, len(segs), sh))
    check(f(fsegs, len(segs), sh))
    res["mixed_4x65536"] = {"ms": ms, "frames_per_s": 4 * 65536 / (ms * 1e-3), "GBs_algorithmic": nbytes / (ms * 1e-3) / 1e9}
    inv = [(t, ops.forward_kinematics(t, lr4, rt4)[0]) for t, lr4, rt4 in segs]
    isegs, ikeep, iouts = ops._inv_segments(inv)
    nb5 = nbytes + sum(65536 * t.num_joints * 32 for t, _ in inv)
    f = lib().rtg_kinematics_multi_f32
    ms = time_events(lambda: f(fsegs, len(segs), isegs, len(inv), sh))
    check(f(fsegs, len(segs), isegs, len(inv), sh))
    res["config5_fk_and_inverse_4x65536"] = {"ms": ms, "frames_per_s": 4 * 65536 / (ms * 1e-3),
                                             "GBs_algorithmic": nb5 / (ms * 1e-3) / 1e9}
    return res


def solvers():
    zp = np.load(os.path.join(G, "zero_pose.npz"))
    B = int(os.environ.get("RTG_BENCH_B", "262144"))
    res = {}
    Tf = topo("vtrdyn_full")
    body, lh, rh, brot = ops.synth_full_body(Tf, B, seed=7, want_rot=True)
    x = torch.from_numpy(synth.synth_upper_body_inputs(4096, 3)).cuda().repeat(B // 4096, 1, 1).contiguous()
    g21 = torch.from_numpy(synth.synth_body21_pose(4096, 4)[1]).cuda().repeat(B // 4096, 1, 1).contiguous()
    cfg = {
        "full_body_pos": (Solver(_lib.SOLVER_FULL_BODY_POS, zp["vtrdyn_full_local_t"], zp["vtrdyn_full_global_t"],
                                 assets.parents("vtrdyn_full"), True), [body, lh, rh]),
        "upper_body": (Solver(_lib.SOLVER_UPPER_BODY, zp["vtrdyn_local_t"], zp["vtrdyn_global_t"],
                              assets.parents("vtrdyn")), [x]),
        "full_body_rot": (Solver(_lib.SOLVER_FULL_BODY_ROT, zp["vtrdyn_full_local_t"], zp["vtrdyn_full_global_t"],
                                 assets.parents("vtrdyn_full")), [brot, body, lh, rh]),
        "body_rot": (Solver(_lib.SOLVER_BODY_ROT, zp["vtrdyn_local_t"], zp["vtrdyn_global_t"],
                            assets.parents("vtrdyn")), [g21]),
    }
    for k, (S, ins) in cfg.items():
        dof = torch.empty((B, 30), device="cuda")
        ms = time_events(lambda: S.retarget(ins, out_dof=dof))
        res[k] = {"ms": ms, "frames_per_s": B / (ms * 1e-3)}
    return res


def aux():
    """The §8(f) kernels around the solver: VTRDyn ingest (23/20/20-point broadcast frames -> solver rows and the
    has-data flag, both layouts) and the SkeletonMotion velocity stencils (gradient + gaussian smoothing), at
    262144 frames.  Algorithmic bytes: ingest 189 floats in + 183 floats + 1 flag out per frame; velocities the
    input and output rows once each (the smoothing's intermediate pass is the kernels' own traffic)."""
    from rtg import ingest
    B = 262144
    res = {}
    g = torch.Generator().manual_seed(5)
    b23 = torch.randn(B, 23, 3, generator=g).cuda()
    l20 = torch.randn(B, 20, 3, generator=g).cuda()
    r20 = torch.randn(B, 20, 3, generator=g).cuda()
    nbytes = B * ((23 + 20 + 20) * 3 * 4 + (21 + 20 + 20) * 3 * 4 + 1)
    for layout in ("aos", "soa"):
        ms = time_events(lambda: ingest.reindex_frames(b23, l20, r20, layout=layout))
        res[f"ingest_{layout}_262144"] = {"ms": ms, "frames_per_s": B / (ms * 1e-3),
                                           "GBs_algorithmic": nbytes / (ms * 1e-3) / 1e9}
    nseq, L, J = 64, 4096, 31   # 64 motions of 4096 frames, Hu links
    p = torch.randn(nseq, L, J, 3, generator=g).cuda()
    q = torch.nn.functional.normalize(torch.randn(nseq, L, J, 4, generator=g), dim=-1).cuda()
    for name, fn, nb in (("linear_velocity", lambda: ops.motion_velocity(p, 1.0 / 30), nseq * L * J * 24),
                         ("angular_velocity", lambda: ops.motion_angular_velocity(q, 1.0 / 30), nseq * L * J * 28)):
        ms = time_events(fn)
        res[f"{name}_64x4096"] = {"ms": ms, "frames_per_s": nseq * L / (ms * 1e-3), "GBs_algorithmic": nb / (ms * 1e-3) / 1e9}
    return res


def sweep():
    """FULL_BODY_POS kernel time across batch sizes (RTG_LATENCY_MAX_B picks the latency kernel below it): run with
    the default library and with an RTG_LATENCY_MAX_B=0 build (RTG_LIB=...) to find the crossover."""
    zp = np.load(os.path.join(G, "zero_pose.npz"))
    S = Solver(_lib.SOLVER_FULL_BODY_POS, zp["vtrdyn_full_local_t"], zp["vtrdyn_full_global_t"],
               assets.parents("vtrdyn_full"), True)
    Tf = topo("vtrdyn_full")
    res = {}
    for B in (256, 1024, 2048, 4096, 8192, 16384, 24576, 32768, 49152, 65536, 98304, 131072):
        body, lh, rh = ops.synth_full_body(Tf, B, seed=7)[:3]
        dof = torch.empty((B, 30), device="cuda")
        ms = time_events(lambda: S.retarget([body, lh, rh], out_dof=dof))
        res[str(B)] = {"kernel_us": ms * 1e3, "frames_per_s": B / (ms * 1e-3)}
    return res


if __name__ == "__main__":
    modes = sys.argv[1:] or ["latency", "fk", "solvers"]
    out = {m: globals()[m]() for m in modes}
    print(json.dumps(out, indent=1))
