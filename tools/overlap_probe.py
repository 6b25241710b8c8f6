"""Does the next batch fill the CUs that the previous batch's last tiles leave idle?  The headline kernel's tiles all
start together, the CU's oldest waves get issue priority, and its last tiles run alone (tools/side_phases.py: round-1
tiles end between 35 and 64 us); a following batch on ANOTHER stream can start its tiles on those CUs.

Times K full solves (FULL_BODY_POS, B = 262144, SoA, ring of input sets) three ways: one stream; two streams
alternating (step i on stream i % 2, every step still one full batched solve); and both captured as HIP graphs.
Prints us per step and checks every step's DOFs equal the single-stream ones.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "humanoid-real-time-retarget_amd"))

from rtg import _lib, assets, ops  # noqa: E402
from rtg.runtime import Solver, Topology  # noqa: E402


def main(K=20, B=262144, R=4):
    zp = np.load(os.path.join(REPO, "tests", "golden", "zero_pose.npz"))
    S = Solver(_lib.SOLVER_FULL_BODY_POS, zp["vtrdyn_full_local_t"], zp["vtrdyn_full_global_t"],
               assets.parents("vtrdyn_full"), True)
    T = Topology(assets.parents("vtrdyn_full"), assets.local_translation("vtrdyn_full"), assets.tree_quat("vtrdyn_full"))
    sets = [ops.synth_full_body(T, B, seed=1234, frame_offset=r * B, layout="soa") for r in range(R)]
    outs = [torch.empty((B, 30), device="cuda") for _ in range(R)]
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]

    def step(i, nstreams):
        s = streams[i % nstreams]
        with torch.cuda.stream(s):
            S.retarget(list(sets[i % R]), out_dof=outs[i % R], layout="soa")

    def timed(nstreams, graph):
        main_s = streams[0]
        run = None
        if graph:
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                cap = torch.cuda.current_stream()
                fork = torch.cuda.Event()
                fork.record(cap)
                side = streams[1]
                side.wait_event(fork)
                for i in range(K):
                    s = cap if (nstreams == 1 or i % 2 == 0) else side
                    with torch.cuda.stream(s):
                        S.retarget(list(sets[i % R]), out_dof=outs[i % R], layout="soa")
                join = torch.cuda.Event()
                join.record(side)
                cap.wait_event(join)
            g.replay()
            torch.cuda.synchronize()
            run = g.replay
        else:
            def run():
                for i in range(K):
                    step(i, nstreams)
                if nstreams > 1:
                    main_s.wait_stream(streams[1])
        res = []
        for _ in range(5):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main_s)
            if nstreams > 1 and not graph:
                streams[1].wait_event(e0)
            run()
            e1.record(main_s)
            e1.synchronize()
            res.append(1e3 * e0.elapsed_time(e1) / K)
        return res

    for i in range(100):   # warm the clocks before any mode is timed
        step(i, 1)
    torch.cuda.synchronize()
    ref = [o.clone() for o in outs]
    out = {"B": B, "K": K, "box": ops.box_probe()}
    modes = (("one_stream", 1, False), ("two_streams", 2, False), ("graph_one_stream", 1, True),
             ("graph_two_streams", 2, True))
    runs = {m[0]: [] for m in modes}
    for rnd in range(3):   # modes interleaved, so clock drift hits each alike
        for name, ns, graph in modes:
            try:
                runs[name] += timed(ns, graph)[1:]
                torch.cuda.synchronize()
                if not all(torch.equal(a, b) for a, b in zip(outs, ref)):
                    runs[name + "_dofs_differ"] = True
            except Exception as e:  # noqa: BLE001
                out[name] = {"error": repr(e)}
    for name, us in runs.items():
        if us and isinstance(us, list):
            out[name] = {"us_min": round(min(us), 2), "us_median": round(float(np.median(us)), 2),
                         "frames_per_s_median": B / (float(np.median(us)) * 1e-6)}
        elif us is True:
            out[name] = True
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
