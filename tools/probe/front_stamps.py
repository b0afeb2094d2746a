#!/usr/bin/env python3
"""Diagnostic: per-phase wall-clock sums of front_solve_kernel (a PBA_FRONT_STAMPS variant writes them over x[0 … 29];
the step it returns is then meaningless).  C3-size free-intrinsics problem, one camera.

    PBA_LIBRARY=variants/libpba_fst.so python3 tools/probe/front_stamps.py
"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
synth = importlib.import_module("photometric-bundle-adjustment_amd.synth")
E = importlib.import_module("photometric-bundle-adjustment_amd.engine")

NAMES = ["loads", "-", "panel", "bar B", "trail|factor+fresh", "bar C", "bwd dot", "bar 1", "bwd solve", "bar 2"]

if __name__ == "__main__":
    nf = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    pb = synth.make_problem(kind="geometric", model="pinhole", n_frames=nf, n_points=100 * nf, K=4, seed=5,
                            with_images=False, obs_sigma=0.5)
    with E.Engine(pb.kind, pb.model, huber_width=1.0) as eng:
        eng.set_problem(pb)
        eng.set_fixed_frames(np.array([0, 1], np.int32))
        eng.set_state(pb.poses, pb.rho)
        eng.set_optimize_intrinsics(True)
        eng.gn_linearize()
        for _ in range(3):
            eng.gn_step(1e-3)
        dp, _ = eng.gn_last_step()
    v = dp.ravel()[:30] * 10.0 / 1e3  # 100 MHz ticks → µs
    ncol = nf + 2
    for w, off in (("lane 0", 0), ("lane 64", 10), ("lane 192", 20)):
        print(w, " ".join(f"{n}={v[off + i] / ncol:.3f}" for i, n in enumerate(NAMES)), "µs/column", flush=True)
