#!/usr/bin/env python3
"""Diagnostic: where the C2 drop-in's Jacobian evaluation exceeds Ceres' floor.  Interleaved runs of
the drop-in (gpu), the floor (the same Solve replaying the drop-in's read-backs from cache-hot staged buffers) and the
floor with the staged buffers flushed from the CPU caches (PBA_FLOOR_COLD=1: the drop-in's read-back arrives by DMA into
memory no core has cached); median Jacobian evaluation per mode, Ceres' own timer.

    python3 tools/probe/c2_floor_probe.py [runs]
"""
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
synth = importlib.import_module("photometric-bundle-adjustment_amd.synth")
import ceres_runner as CR  # noqa: E402


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    threads = int(os.environ.get("PBA_PROBE_THREADS", "16"))
    pb = synth.c2_problem()
    pb.poses[:2] = pb.poses_gt[:2]
    res = {m: [] for m in ("gpu", "floor", "floor_cold")}
    for _ in range(runs):
        for m in res:
            if m == "floor_cold":
                os.environ["PBA_FLOOR_COLD"] = "1"
            r = CR.run("floor" if m.startswith("floor") else "gpu", pb, iters=10, huber=9.0, threads=threads, check=False)
            os.environ.pop("PBA_FLOOR_COLD", None)
            res[m].append(1e3 * r["jacobian_evaluation_s"] / max(r["jacobian_evaluations"], 1))
    for m, v in res.items():
        print(f"{m:10s} median {np.median(v):.3f} ms  min {min(v):.3f}  runs {' '.join(f'{x:.2f}' for x in v)}", flush=True)
    print(f"gpu / floor {np.median(res['gpu']) / np.median(res['floor']):.3f}, gpu / floor_cold "
          f"{np.median(res['gpu']) / np.median(res['floor_cold']):.3f}")


if __name__ == "__main__":
    main()
