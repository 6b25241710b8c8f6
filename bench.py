"""Throughput bench of the batched retarget hot path (BASELINE.json metric).

One step = one launch of VtrdynFullBodyPosRetargeter's batched solver over a
batch of synthetic VTRDyn frames already resident in HBM (BASELINE config 3:
262144 frames per GPU, fp32).  Inputs are generated on the device (seed
1234 + rank) into a ring of buffer sets larger than the 256 MiB Infinity Cache
so every timed step reads cold HBM.  Frames shard across ranks with no
data-path collective ("scaling": "weak"); the RCCL broadcast of the solver
constants happens at setup and the DOF gather after the timed region.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import shutil
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "humanoid-real-time-retarget_amd")
sys.path.insert(0, PKG)
sys.path.insert(0, os.path.join(REPO, "oracle"))

METRIC = "retargeted frames/sec + max joint-angle err vs ref, Hu humanoid @1/2/4/8 GPU"
BYTES_PER_FRAME = 504          # 32 used input points x 12 B + 30 DOF x 4 B
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=262144, help="frames per GPU per step")
    ap.add_argument("--ring", type=int, default=0, help="input buffer sets (0 = enough to exceed 256 MiB x 2)")
    ap.add_argument("--layout", choices=("soa", "aos"), default="soa",
                    help="input layout of the timed frames: SoA component planes as the device producer emits them "
                         "(default, north_star), or the reference's AoS rows; the other one is reported as a "
                         "secondary line")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    return ap.parse_args()


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int) -> int:
    """``--gpus N`` without a launcher: start N fresh rank processes of this script (one per GPU, RANK / LOCAL_RANK
    / WORLD_SIZE / MASTER_* in their environment) and return the first non-zero exit code.  The parent never touches
    the GPU, so each child initialises HIP itself; rank 0 prints the JSON line."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                code = p.poll()
                if code is None:
                    continue
                pending.remove(p)
                if code != 0 and rc == 0:
                    rc = code
                    for q in pending:      # one rank failed: the others would wait in a collective forever
                        q.terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc


def load_backend():
    """The rank backend: DeviceBackend (librtg_hip.so + RCCL) unless RTG_BENCH_BACKEND=module:Class names a stand-in
    (the gloo tests drive this script's own launch path with a host backend)."""
    spec = os.environ.get("RTG_BENCH_BACKEND")
    if not spec:
        return DeviceBackend
    import importlib
    mod, cls = spec.split(":")
    return getattr(importlib.import_module(mod), cls)


def dist_setup(backend_cls):
    """Rank / world from the launcher's environment; the process group over RCCL ("nccl") for the device backend."""
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend_cls.bind_device(local)
    if world > 1:
        dist.init_process_group(backend_cls.DIST_BACKEND, **backend_cls.pg_kwargs(local))
    return world, rank, local


def barrier(world, backend=None):
    """Barrier + device synchronise on both sides of the timed region."""
    if world > 1:
        import torch.distributed as dist
        dist.barrier()
    if backend is not None:
        backend.sync()
    else:
        import torch
        torch.cuda.synchronize()


def rocm_smi_clocks(dev: int):
    """Current sclk / mclk as rocm-smi reports them for this device (None when rocm-smi is unavailable)."""
    if "rocprof" in os.environ.get("LD_PRELOAD", ""):
        return None   # under rocprofv3 a child process would initialise the GPU through the profiler's preload
    try:
        # the script through this interpreter: no `#!/usr/bin/env` hop (an exec) in the child
        smi = os.path.realpath(shutil.which("rocm-smi") or "/opt/rocm/bin/rocm-smi")
        r = subprocess.run([sys.executable, smi, "-d", str(dev), "--showclocks", "--json"], capture_output=True,
                           text=True, timeout=30)
        card = next(iter(json.loads(r.stdout).values()))
        return {k: v for k, v in card.items() if "sclk" in k or "mclk" in k}
    except Exception:  # noqa: BLE001
        return None


def cpu_share() -> int:
    """CPUs this process may use: the affinity mask, capped by a cgroup v2 CPU quota (the GPU box exposes the
    whole machine in os.cpu_count() but grants one GPU's share of it)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return max(1, n)


_PER_FRAME_CHILD = r"""
import os, sys, time, numpy as np
sys.path.insert(0, sys.argv[1])
import oracle as orc
orc.lib().oracle_set_threads(1)
d = np.load(sys.argv[2])
lo, hi, secs = int(sys.argv[3]), int(sys.argv[4]), float(sys.argv[5])
b, l, r, zl, zg = d["body"][lo:hi], d["lh"][lo:hi], d["rh"][lo:hi], d["zl"], d["zg"]
done, t0 = 0, time.perf_counter()
while time.perf_counter() - t0 < secs:
    for i in range(0, hi - lo, 64):   # 64-frame calls of the per-frame C solver, one core
        orc.full_body_pos(zl, zg, b[i:i + 64], l[i:i + 64], r[i:i + 64], True, want_rot=False)
        done += min(64, hi - lo - i)
print(done, time.perf_counter() - t0)
"""


def cpu_baseline(body, lh, rh, zl, zg, seconds):
    """The oracle (the C port of the reference path, kind "port") on the host's CPU share, bounded sample:
    (1) the batched path, OpenMP over every CPU of the share (thread count pinned through the oracle);
    (2) SURVEY §8d's per-frame leg: one single-thread process per CPU of the share on disjoint frame slices.
    The GPU box's os.cpu_count() is the whole machine; this job is granted a share of it (cpu_share())."""
    import tempfile

    import oracle as orc
    share = cpu_share()
    lib = orc.lib()
    lib.oracle_set_threads(share)
    threads = int(lib.oracle_max_threads())
    n = body.shape[0]
    orc.full_body_pos(zl, zg, body[:256], lh[:256], rh[:256], True, want_rot=False)   # warm
    done, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        orc.full_body_pos(zl, zg, body, lh, rh, True, want_rot=False)
        done += n
    dt = time.perf_counter() - t0
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:  # noqa: BLE001
        model = "unknown"
    out = {"value": done / dt, "unit": "frames/s", "cores": threads, "kind": "port",
           "sample": f"{done} synthetic frames ({n}-frame slices of the bench workload), oracle/rtg_oracle.c "
                     f"OpenMP x{threads}, {dt:.1f} s", "cpu": model, "host_cpus": os.cpu_count(), "cpu_share": share,
           "per_core_frames_per_s": done / dt / threads,
           "reference_python_cross_ref": {
               "frames_per_s": 216.0, "ms_per_frame": 4.63, "cores": 1,
               "cpu": "8-vCPU Intel Xeon (AVX-512) build container, torch 2.10.0 CPU, MKL 2024.2",
               "code": "VtrdynFullBodyPosRetargeter.retarget (full_body_pos_retargeter.py:25-59), 1 process x 1 thread",
               "source": "BASELINE.md:25 / SURVEY.md section 6 (measured there, not in this run: the reference's "
                         "Python cannot travel to the GPU box)"}}
    # per-frame leg: `share` independent single-thread processes (children never touch the GPU)
    try:
        with tempfile.TemporaryDirectory() as td:
            path = os.path.join(td, "frames.npz")
            np.savez(path, body=body, lh=lh, rh=rh, zl=zl, zg=zg)
            per = n // share
            secs = max(2.0, seconds / 2)
            procs = [subprocess.Popen([sys.executable, "-c", _PER_FRAME_CHILD, os.path.join(REPO, "oracle"), path,
                                       str(k * per), str((k + 1) * per), str(secs)], stdout=subprocess.PIPE,
                                      stderr=subprocess.DEVNULL, env=dict(os.environ, OMP_NUM_THREADS="1"), text=True)
                     for k in range(share)]
            res = [p.communicate(timeout=secs * 4 + 60)[0].split() for p in procs]
            frames = sum(int(r[0]) for r in res)
            rate = sum(int(r[0]) / float(r[1]) for r in res)
            out["per_frame_processes"] = {"processes": share, "frames_per_s": rate, "frames": frames,
                                          "us_per_frame_per_process": share / rate * 1e6,
                                          "sample": f"{per}-frame slice per process, {secs:.0f} s each"}
    except Exception as e:  # noqa: BLE001
        out["per_frame_processes"] = {"error": repr(e)}
    return out


PMC_JSON = os.path.join(REPO, "profiles", "pmc_r06.json")
PMC_KERNELS = {"soa": "rtg::k_solve_sides<0, true, true>", "aos": "rtg::k_solve_sides<0, true, false>"}
VALU_PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9   # MI355X: CUs x SIMDs x lanes issued per cycle x 2.4 GHz (78.6 T/s)


def pmc_record(B, layout="soa"):
    """The committed rocprofv3 PMC summary of the headline kernel (tools/profile_round.sh -> tools/pmc_summary.py),
    when it was taken at this batch (rocprofv3's grid counts threads: two per frame, one wave per side)."""
    try:
        rec = json.load(open(PMC_JSON)).get(PMC_KERNELS[layout])
    except (OSError, ValueError):
        return None
    if not rec or rec.get("grid") != 2 * B:
        return None
    return rec


def compute_roofline(rec, kern_ms):
    """VALU side of the roofline: the kernel's VALU instructions per launch (SQ_INSTS_VALU, PMC) x 64 lanes over the
    measured kernel time, against the 78.6 T lane-op/s issue peak; `frac_issue_weighted` charges f64 ops 2 issue
    slots and transcendentals 4 (f32) / 8 (f64) -- the cycle cost the kernel actually pays."""
    if not rec or "valu_insts" not in rec:
        return None
    t = kern_ms * 1e-3
    achieved = rec["valu_insts"] * 64 / t
    return {"bound": "valu", "achieved": achieved / 1e12, "peak": VALU_PEAK_LANE_OPS / 1e12, "unit": "T lane-ops/s",
            "frac": achieved / VALU_PEAK_LANE_OPS,
            "frac_issue_weighted": rec["valu_issue_weighted"] * 64 / t / VALU_PEAK_LANE_OPS,
            "valu_wave_insts_per_launch": rec["valu_insts"],
            "valu_lane_ops_per_frame": rec["valu_insts"] * 64 / (rec["grid"] / 2)}


def secondary_configs(solver, sets, stream):
    """BASELINE configs 2 and 5 on the same GPU (reported beside the headline line, not as `value`):
    config 2 = 4096 frames per launch (latency-bound regime), kernel-only and PCIe-inclusive (pinned host
    frames in, DOFs back); config 5 = FK plus inverse FK of 4 robot_config skeletons x 65536 frames, one launch."""
    import torch
    from rtg import assets, ops, synth
    from rtg.runtime import Topology
    out = {}
    n = 4096
    xb, xl, xr = sets   # 4096 AoS frames (the per-frame callers' rows)
    d = torch.empty((n, 30), device=xb.device)
    for _ in range(10):
        solver.retarget([xb, xl, xr], out_dof=d)
    # timed through the C ABI with the arguments built once: Solver.retarget's checks cost ~15-20 us of host time
    # per call, about the kernel's own, so back-to-back Python calls would time the host
    from rtg import _lib
    from rtg._lib import lib
    from rtg.runtime import ptr, stream_handle
    args = (solver.handle, ptr(xb), ptr(xl), ptr(xr), None, n, _lib.LAYOUT_AOS, ptr(d), None, None,
            stream_handle(stream))
    launch = lib().rtg_retarget_f32
    reps = 200
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        launch(*args)
    e1.record(stream)
    e1.synchronize()
    k_ms = e0.elapsed_time(e1) / reps
    hb, hl, hr = (t.cpu().pin_memory() for t in (xb, xl, xr))
    hd = torch.empty((n, 30)).pin_memory()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        xb.copy_(hb, non_blocking=True); xl.copy_(hl, non_blocking=True); xr.copy_(hr, non_blocking=True)
        solver.retarget([xb, xl, xr], out_dof=d)
        hd.copy_(d, non_blocking=True)
        torch.cuda.synchronize()
    e2e_ms = (time.perf_counter() - t0) * 1e3 / 50
    out["config2_batch4096"] = {"kernel_ms": k_ms, "frames_per_s": n / (k_ms * 1e-3), "e2e_pcie_ms": e2e_ms,
                                "e2e_pcie_frames_per_s": n / (e2e_ms * 1e-3)}
    fk, inv, nbytes = [], [], 0
    for i, name in enumerate(["hu_v5", "vtrdyn", "vtrdyn_full", "noitom"]):
        t = Topology(assets.parents(name), assets.local_translation(name), assets.tree_quat(name))
        J = t.num_joints
        lr = torch.from_numpy(synth.random_local_quats(65536, J, 10 + i)).cuda()
        fk.append((t, lr, torch.zeros((65536, 3), device="cuda")))
        nbytes += 65536 * (J * 16 + 12 + J * 28)        # FK: local rotations + root in, rotations + positions out
        inv.append((t, ops.forward_kinematics(t, lr, torch.zeros((65536, 3), device="cuda"))[0]))
        nbytes += 65536 * (J * 16 + J * 16)             # inverse FK: global rotations in, local rotations out
    # the segment tables and outputs built once, the launch through the C ABI: ops.kinematics_multi allocates its
    # outputs per call, and that host time (~0.1 ms) would be what back-to-back calls measure
    from rtg._lib import check, lib
    from rtg.runtime import stream_handle
    fsegs, fkeep, fouts = ops._fk_segments(fk)
    isegs, ikeep, iouts = ops._inv_segments(inv)
    launch, sh = lib().rtg_kinematics_multi_f32, stream_handle(stream)
    for _ in range(5):
        check(launch(fsegs, len(fk), isegs, len(inv), sh))
    e0.record(stream)
    for _ in range(50):
        launch(fsegs, len(fk), isegs, len(inv), sh)
    e1.record(stream)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / 50
    out["config5_mixed_fk_and_inverse_4x65536"] = {
        "kernel_ms": ms, "frames_per_s": 4 * 65536 / (ms * 1e-3), "GBs_algorithmic": nbytes / (ms * 1e-3) / 1e9,
        "hbm_frac": nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
        "launch": "rtg_kinematics_multi_f32: 4 FK + 4 inverse-FK segments in one launch"}
    return out


def layout_line(solver, topo_full, B, rank, ring, steps, stream, layout):
    """The same workload in the other input layout, reported beside the headline (not as `value`):
    AoS = the reference's (B, P, 3) rows, each wave load of a point a 64-line gather of 12-byte pieces;
    SoA = (P, C, B) component planes emitted directly by the device producer, each load 256 contiguous bytes."""
    import torch
    from rtg import ops
    sets = []
    for r in range(ring):
        b, l, r_ = ops.synth_full_body(topo_full, B, seed=1234 + rank, frame_offset=r * B, layout=layout)
        sets.append((b, l, r_, torch.empty((B, 30), device=b.device)))
    for i in range(5):
        b, l, r_, d = sets[i % ring]
        solver.retarget([b, l, r_], out_dof=d, layout=layout)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for i in range(steps):
        b, l, r_, d = sets[i % ring]
        solver.retarget([b, l, r_], out_dof=d, layout=layout)
    e1.record(stream)
    e1.synchronize()
    ms = e0.elapsed_time(e1) / steps
    gbs = BYTES_PER_FRAME * B / (ms * 1e-3) / 1e9
    return {"layout": layout, "kernel_ms": ms, "frames_per_s": B / (ms * 1e-3), "achieved_GBs": gbs,
            "hbm_frac": gbs / HBM_PEAK_GBS, "input_ring_sets": ring}


def parity_vs_reference():
    """max / p99 |dof_gpu - dof_ref| on the committed reference golden vectors."""
    import torch
    from rtg import _lib, assets
    from rtg.runtime import Solver
    g = np.load(os.path.join(REPO, "tests", "golden", "full_body_pos_precise.npz"))
    zp = np.load(os.path.join(REPO, "tests", "golden", "zero_pose.npz"))
    S = Solver(_lib.SOLVER_FULL_BODY_POS, zp["vtrdyn_full_local_t"], zp["vtrdyn_full_global_t"],
               assets.parents("vtrdyn_full"), True)
    dof, _, _ = S.retarget([torch.from_numpy(np.ascontiguousarray(g[k])).cuda() for k in ("body", "lh", "rh")])
    e = np.abs(dof.cpu().numpy().astype(np.float64) - g["dof"])
    fm = e.max(1)
    out = {"frames": int(len(fm)), "max_abs_err": float(e.max()), "p99_frame_err": float(np.quantile(fm, 0.99)),
           "median_frame_err": float(np.median(fm)), "frac_frames_le_1e-5": float(np.mean(fm <= 1e-5)),
           "unit": "rad (DOFs 18,19,27,28: m)"}
    # the reference against itself: same inputs, MKL forced to another ISA (tools/ref_isa_spread.py)
    sp = np.load(os.path.join(REPO, "tests", "golden", "ref_isa_spread.npz"))
    for isa in sp["isas"]:
        r = np.abs(sp[f"full_body_pos_precise_{isa}"].astype(np.float64) - g["dof"]).max(1)
        out[f"reference_self_spread_mkl_{isa}"] = {"max_abs_err": float(r.max()),
                                                   "p99_frame_err": float(np.quantile(r, 0.99)),
                                                   "frac_frames_le_1e-5": float(np.mean(r <= 1e-5))}
    return out


def source_setup():
    """Rank 0's inputs to the setup broadcast: the VTRDYN_FULL source skeleton (parents, local translations,
    tree quaternions) from the package assets."""
    from rtg import assets
    return (assets.parents("vtrdyn_full"), assets.local_translation("vtrdyn_full"), assets.tree_quat("vtrdyn_full"))


GOLDEN = os.path.join(REPO, "tests", "golden", "full_body_pos_precise.npz")


def golden_errors(dof, gold_dof):
    """max |dof - golden| over the reference's 512 golden frames and the share of frames within 1e-5."""
    e = np.abs(np.asarray(dof, np.float64) - gold_dof).max(1)
    return {"frames": int(len(e)), "max_abs_err": float(e.max()), "frac_frames_le_1e-5": float(np.mean(e <= 1e-5))}


class DeviceBackend:
    """The product path of one rank: librtg_hip.so on this rank's GPU (RCCL for the collectives)."""
    DIST_BACKEND = "nccl"
    DEVICE = True

    @staticmethod
    def bind_device(local):
        import torch
        torch.cuda.set_device(local)

    @staticmethod
    def pg_kwargs(local):
        import torch
        return {"device_id": torch.device("cuda", local)}

    def __init__(self, local, layout="soa"):
        import torch
        self.torch = torch
        self.dev = torch.device("cuda", local)
        self.layout = layout
        self.comm_device = self.dev
        self.stream = torch.cuda.current_stream()
        # RTG_BENCH_STREAMS=2 (default): step i runs on stream i % 2, so the next batch's tiles take the CUs that the
        # previous batch's last tiles leave idle (tools/overlap_probe.py); every step is still one full batched solve
        self.nstreams = max(1, int(os.environ.get("RTG_BENCH_STREAMS", "2")))
        self.streams = [self.stream] + [torch.cuda.Stream(self.dev) for _ in range(self.nstreams - 1)]

    def golden_check(self, solver):
        """This rank's own solver on the reference's golden frames (AoS rows, as the teleop callers hand them)."""
        g = np.load(GOLDEN)
        dof, _, _ = solver.retarget([self.torch.from_numpy(np.ascontiguousarray(g[k])).to(self.dev)
                                     for k in ("body", "lh", "rh")])
        return golden_errors(dof.cpu().numpy(), g["dof"])

    def zero_global(self, parents, lt, tq):
        """The source zero pose's global translations (SkeletonState FK of the identity pose, on the device)."""
        from rtg import ops
        from rtg.runtime import Topology
        T = Topology(parents, lt, tq)
        J = len(parents)
        ident = self.torch.tensor([[0, 0, 0, 1.0]]).expand(1, J, 4)
        return ops.forward_kinematics(T, ident, self.torch.zeros(1, 3), state=True)[1][0].cpu().numpy()

    def build(self, parents, lt, tq, zg):
        from rtg import _lib
        from rtg.runtime import Solver, Topology
        return Topology(parents, lt, tq), Solver(_lib.SOLVER_FULL_BODY_POS, lt, zg, parents, precise_gripper=True)

    def synth(self, topo, B, seed, offset):
        from rtg import ops
        return ops.synth_full_body(topo, B, seed=seed, frame_offset=offset, layout=self.layout)

    def new_dof(self, B):
        return self.torch.empty((B, 30), device=self.dev, dtype=self.torch.float32)

    def solve(self, solver, b, l, r, d):
        solver.retarget([b, l, r], out_dof=d, layout=self.layout)

    def prepare_steps(self, solver, sets, steps):
        """The K timed solves (ring set i % R for step i) captured once, before the timed region, as ONE HIP graph:
        replaying it launches the K kernels back to back without K host-side launch calls (RTG_BENCH_GRAPH=0: plain
        launches).  Every step still runs one full batched solve on its own input set."""
        self.graph = None
        self.settle = self.settle_clocks(solver, sets, steps)
        if self.nstreams > 1:
            return   # two streams: plain launches (measured 95.8 vs 97.8 us/step for the two-stream graph)
        if os.environ.get("RTG_BENCH_GRAPH", "1") == "0":
            return
        torch = self.torch
        try:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for i in range(steps):
                    b, l, r_, d = sets[i % len(sets)]
                    self.solve(solver, b, l, r_, d)
            g.replay()   # the graph's first replay uploads it: keep that out of the timed region
            torch.cuda.synchronize()
            self.graph = g
        except Exception as e:  # noqa: BLE001 -- capture unsupported: time the plain launches
            print(f"bench.py: HIP graph capture failed ({e!r}); timing plain launches", file=sys.stderr)
            self.graph = None

    def settle_clocks(self, solver, sets, steps, min_ms=None):
        """Untimed solves in the timed region's own launch pattern until the GPU runs at its sustained speed: a box
        fresh from idle ramps up over its first ~100 launches (one stream: 115.8 -> 109.6 us per step over 100
        solves; two streams: 385 -> 104 us, tools/overlap_probe.py), and a short --warmup would time that ramp, not
        the kernel.  Runs blocks of K steps for at least RTG_BENCH_SETTLE_MS (default 200) ms of GPU time and
        records each block's per-step time in the line (`settle`)."""
        torch = self.torch
        min_ms = float(os.environ.get("RTG_BENCH_SETTLE_MS", "200")) if min_ms is None else min_ms
        blocks, total = [], 0.0
        while total < min_ms and len(blocks) < 200:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(self.stream)
            self.run_steps(solver, sets, steps)
            e1.record(self.stream)
            e1.synchronize()
            ms = e0.elapsed_time(e1)
            total += ms
            blocks.append(round(1e3 * ms / steps, 2))
        return {"blocks_of_K_steps": len(blocks), "gpu_ms": round(total, 1),
                "us_per_step_first_blocks": blocks[:3], "us_per_step_last_blocks": blocks[-3:]}

    def run_steps(self, solver, sets, steps):
        if self.graph is not None:
            self.graph.replay()
            return
        torch = self.torch
        for s in self.streams[1:]:
            s.wait_stream(self.stream)   # nothing on a side stream starts before the timed region does
        for i in range(steps):
            b, l, r_, d = sets[i % len(sets)]
            with torch.cuda.stream(self.streams[i % self.nstreams]):
                self.solve(solver, b, l, r_, d)
        for s in self.streams[1:]:
            self.stream.wait_stream(s)   # the stop event covers every stream's steps

    def launch_ms(self, solver, sets, n=10):
        """One launch's own duration: an event pair around n back-to-back launches on ONE stream, right after the
        timed region (the roofline's kernel time; with two streams the timed steps overlap, so the per-step time
        over the timed region is shorter than a launch)."""
        torch = self.torch
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(self.stream)
        for i in range(n):
            b, l, r_, d = sets[i % len(sets)]
            self.solve(solver, b, l, r_, d)
        e1.record(self.stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / n

    def sync(self):
        self.torch.cuda.synchronize()

    def identity(self):
        """This rank's GPU: PCI address, UUID, name (rank_flow gathers them and refuses two ranks on one device)."""
        p = self.torch.cuda.get_device_properties(self.dev)
        return {"local_rank": self.dev.index, "name": p.name, "arch": p.gcnArchName,
                "pci": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}", "uuid": str(p.uuid)}

    def probe(self):
        """rtg_box_probe: the shader clock under load, f32 FMA rate and HBM copy bandwidth of this GPU right now,
        plus the clocks rocm-smi reports (kept in the line so numbers from different boxes can be compared)."""
        from rtg import ops
        rec = ops.box_probe()
        rec["rocm_smi"] = rocm_smi_clocks(self.dev.index)
        return rec

    def start(self):
        # kernel time: one HIP event pair around the K launches on the launch stream (a pair per launch would add
        # each event's own packet and cache release to every launch, ~10 us, which rocprofv3's trace does not see)
        self._e0 = self.torch.cuda.Event(enable_timing=True)
        self._e1 = self.torch.cuda.Event(enable_timing=True)
        self._e0.record(self.stream)

    def stop(self):
        self._e1.record(self.stream)

    def elapsed_ms(self):
        self._e1.synchronize()
        return self._e0.elapsed_time(self._e1)


def rank_devices(world, rank, backend):
    """Every rank's device identity (backend.identity(): PCI address, UUID, name), gathered to all ranks before the
    timed region.  With one GPU per rank (the device backend) the identities must be distinct: two ranks on one
    device would report twice the work of one GPU, so EVERY rank raises (none is left waiting in a collective).
    Backends that share a device on purpose (the one-GPU rehearsal) set SHARES_DEVICE."""
    ident = getattr(backend, "identity", None)
    if ident is None:
        return None
    me = dict(ident(), rank=rank)
    if world == 1:
        return [me]
    import torch.distributed as dist
    devices = [None] * world
    dist.all_gather_object(devices, me)
    keys = [(d["pci"], d.get("uuid")) for d in devices]
    if len(set(keys)) != world and not getattr(backend, "SHARES_DEVICE", False):
        raise RuntimeError(f"bench.py: {world} ranks on {len(set(keys))} distinct devices: {devices}")
    return devices


def comm_info(world, backend):
    """The collective library the ranks ran over: torch.distributed's backend and, on the device path, RCCL's
    version (torch's "nccl" backend is RCCL on ROCm)."""
    info = {"world": world, "backend": None, "rccl_version": None}
    if world > 1:
        import torch.distributed as dist
        info["backend"] = dist.get_backend()
    if getattr(backend, "DEVICE", False):
        try:
            import torch
            info["rccl_version"] = ".".join(str(v) for v in torch.cuda.nccl.version())
        except Exception as e:  # noqa: BLE001 -- reported, never fatal
            info["rccl_version"] = repr(e)
    return info


def rank_flow(world, rank, backend, B, steps, warmup, ring):
    """One rank of the bench: setup broadcast -> own shard of B frames generated locally (seed
    1234 + rank) -> K timed solves between barriers -> max over ranks -> untimed DOF gather to rank 0."""
    from rtg import shard
    setup = None
    if rank == 0:
        parents, lt, tq = source_setup()
        setup = (parents, lt, tq, backend.zero_global(parents, lt, tq))
    if world > 1:   # topology + zero pose from rank 0: the other ranks read no assets
        parents, lt, tq, zg = shard.broadcast_setup(setup, max_joints=64, device=backend.comm_device)
    else:
        parents, lt, tq, zg = setup
    topo, solver = backend.build(parents, lt, tq, zg)
    devices = rank_devices(world, rank, backend)
    sets = []
    for r in range(ring):
        b, l, r_ = backend.synth(topo, B, 1234 + rank, r * B)
        sets.append((b, l, r_, backend.new_dof(B)))
    backend.sync()
    probe = getattr(backend, "probe", None)   # the box's clock and bandwidth, measured before the timed region
    box = {"before": probe()} if probe is not None else None
    for i in range(warmup):
        b, l, r_, d = sets[i % ring]
        backend.solve(solver, b, l, r_, d)
    prepare = getattr(backend, "prepare_steps", None)   # the device backend captures the K steps as one HIP graph
    if prepare is not None:
        prepare(solver, sets, steps)
    barrier(world, backend)
    t0 = time.perf_counter()
    backend.start()
    run = getattr(backend, "run_steps", None)
    if run is not None:
        run(solver, sets, steps)
    else:
        for i in range(steps):
            b, l, r_, d = sets[i % ring]
            backend.solve(solver, b, l, r_, d)
    backend.stop()
    barrier(world, backend)
    wall = time.perf_counter() - t0
    gpu_step_ms = backend.elapsed_ms() / max(1, steps)
    launch = getattr(backend, "launch_ms", None)
    kern_ms = launch(solver, sets) if launch is not None else gpu_step_ms
    kern_ms_rank = kern_ms
    if world > 1:   # the bench clock and the kernel clock are both the slowest rank's
        wall = shard.max_over_ranks(wall, backend.comm_device)
        kern_ms = shard.max_over_ranks(kern_ms, backend.comm_device)
    # every rank checks its own device solver against the reference goldens (after the timed region)
    gold = backend.golden_check(solver)
    per_rank = [gold]
    if world > 1:
        vals = shard.all_gather_floats([gold["max_abs_err"], gold["frac_frames_le_1e-5"], kern_ms_rank],
                                       backend.comm_device)
        per_rank = [{"rank": r, "frames": gold["frames"], "max_abs_err": v[0], "frac_frames_le_1e-5": v[1],
                     "kern_ms": v[2]} for r, v in enumerate(vals)]
    if box is not None:
        box["after"] = probe()
    out = {"wall": wall, "kern_ms": kern_ms, "gpu_step_ms": gpu_step_ms, "frames": world * B * steps, "sets": sets, "topo": topo,
           "solver": solver, "zl": lt, "zg": zg, "parents": parents, "golden_per_rank": per_rank, "box": box,
           "devices": devices, "comm": comm_info(world, backend)}
    if world > 1:   # final DOF gather to rank 0 (untimed region, reported separately)
        d = sets[(steps - 1) % ring][3]
        backend.sync()
        tg = time.perf_counter()
        out["gathered"] = shard.gather_shards(d, [B] * world, dst=0)
        backend.sync()
        out["gather_ms"] = (time.perf_counter() - tg) * 1e3
    return out


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if world_env is not None and int(world_env) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={world_env}", file=sys.stderr)
        sys.exit(2)
    backend_cls = load_backend()
    world, rank, local = dist_setup(backend_cls)
    if not getattr(backend_cls, "DEVICE", False):   # (a subclass may come from `import bench`, not __main__)
        return host_main(args, backend_cls(local), world, rank)
    B = args.batch
    backend = backend_cls(local, args.layout)
    bytes_per_set = B * (63 + 60 + 60 + 30) * 4
    ring = args.ring or max(2, int(np.ceil(2 * 256 * 2**20 / bytes_per_set)))
    res = rank_flow(world, rank, backend, B, args.steps, args.warmup, ring)
    wall, kern_ms = res["wall"], res["kern_ms"]
    value = res["frames"] / wall
    ms_per_step = wall * 1e3 / args.steps
    stream = backend.stream
    if rank == 0:
        achieved = BYTES_PER_FRAME * B / (kern_ms * 1e-3) / 1e9
        rec = pmc_record(B, args.layout)
        line = {
            "metric": METRIC, "value": value, "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic (device-generated VTRDyn frames, seed 1234+rank)",
            "config": {"workload": "VtrdynFullBodyPosRetargeter batched solve, Hu v5 target (BASELINE config 3)",
                       "frames_per_gpu_per_step": B, "global_batch": B * world, "parallelism": f"dp{world}",
                       "input_layout": args.layout, "input_ring_sets": ring, "precise_gripper": True,
                       "launch": "one HIP graph of the K solves" if getattr(backend, "graph", None) is not None
                       else (f"K plain launches, step i on stream i % {backend.nstreams}" if backend.nstreams > 1
                             else "K plain launches")},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": rec["traffic_bytes"] if rec else None,
                         "kernel": f"k_solve_sides<FULL_BODY_POS, {args.layout.upper()}>", "kernel_ms": kern_ms,
                         "kernel_ms_source": "event pair around 10 single-stream launches right after the timed region",
                         "gpu_ms_per_step": res["gpu_step_ms"],
                         # the same bytes over the timed region's per-step GPU time (steps overlap on two streams)
                         "achieved_per_step": BYTES_PER_FRAME * B / (res["gpu_step_ms"] * 1e-3) / 1e9,
                         "frac_per_step": BYTES_PER_FRAME * B / (res["gpu_step_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "bytes_per_frame": BYTES_PER_FRAME,
                         "traffic_unit": "bytes/launch (rocprofv3 FETCH_SIZE x calibration + WRITE_SIZE)",
                         "traffic_detail": {k: rec[k] for k in ("fetch_size_raw", "fetch_correction", "fetch_bytes",
                                                                "write_bytes", "angle_table_fetch_bytes") if k in rec}
                         if rec else None,
                         "compute": compute_roofline(rec, kern_ms)},
        }
        line["settle"] = getattr(backend, "settle", None)
        line["golden_per_rank"] = res["golden_per_rank"]
        line["devices"] = res["devices"]   # one entry per rank: distinct PCI addresses (checked in rank_flow)
        line["comm"] = res["comm"]
        line["box"] = res["box"]
        if "gather_ms" in res:
            line["gather_ms"] = res["gather_ms"]
        from rtg import ops
        aos = ops.synth_full_body(res["topo"], min(B, 65536), seed=1234 + rank)   # rows for config 2 / the CPU leg
        if world == 1:
            solver, sets = res["solver"], res["sets"]
            try:
                line["secondary"] = secondary_configs(solver, [t[:4096].contiguous() for t in aos], stream)
            except Exception as e:  # noqa: BLE001
                line["secondary"] = {"error": repr(e)}
            other = "aos" if args.layout == "soa" else "soa"
            try:
                del sets[:]
                line["secondary"][f"config3_{other}_layout"] = layout_line(solver, res["topo"], B, rank, ring,
                                                                           args.steps, stream, other)
            except Exception as e:  # noqa: BLE001
                line["secondary"][f"config3_{other}_layout"] = {"error": repr(e)}
        try:
            line["parity_vs_reference"] = parity_vs_reference()
        except Exception as e:  # noqa: BLE001
            line["parity_vs_reference"] = {"error": repr(e)}
        if world == 1 and not args.no_cpu_baseline:
            b, l, r_ = aos
            line["cpu_baseline"] = cpu_baseline(b.cpu().numpy(), l.cpu().numpy(), r_.cpu().numpy(),
                                                np.asarray(res["zl"], np.float32), np.asarray(res["zg"], np.float32),
                                                args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def host_main(args, backend, world, rank):
    """The launch/collective flow with a stand-in backend (tests): same rank_flow, a reduced line."""
    res = rank_flow(world, rank, backend, args.batch, args.steps, args.warmup, max(2, args.ring))
    if rank == 0:
        line = {"metric": METRIC, "value": res["frames"] / res["wall"], "unit": "frames/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "backend": type(backend).__name__,
                "kern_ms": res["kern_ms"], "golden_per_rank": res["golden_per_rank"], "devices": res["devices"],
                "comm": res["comm"]}
        if "gathered" in res:
            line["gathered_sha1"] = hashlib.sha1(res["gathered"].numpy().tobytes()).hexdigest()
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
