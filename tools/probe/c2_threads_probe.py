#!/usr/bin/env python3
"""Diagnostic: does the C2 drop-in lose its Jacobian evaluations to the process's CPU quota?  Ceres
runs 16 threads on a 16-CPU cgroup quota; the drop-in adds the HIP runtime's threads (and its chunk waits) on top.
Interleaved runs of the drop-in with 16 and 15 Ceres threads and of the replay floor with 16, median Jacobian evaluation
per mode (Ceres' own timer), and the cgroup's throttling counters (cpu.stat: nr_throttled, throttled_usec) over each run.

    python3 tools/probe/c2_threads_probe.py [runs]
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


def cpu_stat():
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            return {k: int(v) for k, v in (line.split() for line in f if len(line.split()) == 2)}
    except OSError:
        return {}


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 7
    pb = synth.c2_problem()
    pb.poses[:2] = pb.poses_gt[:2]
    modes = [("gpu", 16), ("gpu", 15), ("gpu", 14), ("floor", 16)]
    res = {m: [] for m in modes}
    thr = {m: [] for m in modes}
    for _ in range(runs):
        for m in modes:
            s0 = cpu_stat()
            r = CR.run(m[0], pb, iters=10, huber=9.0, threads=m[1], check=False)
            s1 = cpu_stat()
            res[m].append(1e3 * r["jacobian_evaluation_s"] / max(r["jacobian_evaluations"], 1))
            thr[m].append((s1.get("nr_throttled", 0) - s0.get("nr_throttled", 0),
                           (s1.get("throttled_usec", 0) - s0.get("throttled_usec", 0)) / 1e3))
    floor = np.median(res[("floor", 16)])
    for m, v in res.items():
        t = np.array(thr[m])
        print(f"{m[0]:5s} {m[1]:2d} threads: median {np.median(v):.3f} ms (x{np.median(v) / floor:.3f} of the floor)  "
              f"runs {' '.join(f'{x:.2f}' for x in v)}  throttled periods {int(t[:, 0].sum())}, "
              f"{t[:, 1].sum():.1f} ms", flush=True)
    print("cpu.stat keys:", sorted(cpu_stat()))


if __name__ == "__main__":
    main()
