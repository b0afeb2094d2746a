#!/usr/bin/env python3
"""Diagnostic: the free-intrinsics border kernels (intr_rows_kernel, intr_border_kernel) at C3 and C4 sizes —
geometric engines (reprojection functor), pba_solve with set_optimize_intrinsics, one and two cameras.  Run under
`rocprofv3 --kernel-trace --stats`; prints ms per LM iteration of each case.

    rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/intr -o run -- python3 tools/probe/intr_probe.py
"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
synth = importlib.import_module("photometric-bundle-adjustment_amd.synth")
E = importlib.import_module("photometric-bundle-adjustment_amd.engine")


def run(tag, n_frames, n_points, cams):
    fc = None if cams == 1 else (np.arange(n_frames) % cams).astype(np.int32)
    intr = None
    if cams > 1:
        base = synth.make_problem(kind="geometric", model="pinhole", n_frames=8, n_points=8, with_images=False).intrinsics
        intr = np.repeat(base[:1], cams, axis=0) * np.linspace(0.99, 1.01, cams)[:, None] ** np.array([1, 1, 0, 0, 0, 0, 0, 0])
    pb = synth.make_problem(kind="geometric", model="pinhole", n_frames=n_frames, n_points=n_points, K=4, seed=5,
                            with_images=False, frame_cam=fc, intrinsics=intr, obs_sigma=0.5)
    pb.poses[:2] = pb.poses_gt[:2]
    with E.Engine(pb.kind, pb.model, huber_width=1.0) as eng:
        eng.set_problem(pb)
        eng.set_fixed_frames(np.array([0, 1], np.int32))
        eng.set_state(pb.poses, pb.rho)
        eng.set_optimize_intrinsics(True)
        eng.solve(max_iterations=2)
        eng.set_state(pb.poses, pb.rho)
        s = eng.solve(max_iterations=10, function_tolerance=0.0)
    print(f"{tag}: {pb.n_blocks} blocks, {cams} camera(s): {s['total_ms'] / max(s['iterations'], 1):.3f} ms per LM "
          f"iteration, {s['successful_steps']}/{s['unsuccessful_steps']}", flush=True)


if __name__ == "__main__":
    run("C3", 200, 20000, 1)
    run("C3", 200, 20000, 2)
    run("C4", 1000, 100000, 1)
