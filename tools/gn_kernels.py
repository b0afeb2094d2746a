#!/usr/bin/env python3
"""Diagnostic: the GN kernels of one LM iteration at C4, run unconditionally (linearise, step, candidate cost) N
times at a fixed state, for `rocprofv3 --kernel-trace --stats` per-kernel averages of a library variant
(PBA_LIBRARY=…).  Not a parity check and not the bench: variants under study may compute garbage.

    rocprofv3 --kernel-trace --stats -d gpurun_out/gnk -o run -- python tools/gn_kernels.py [--iters 20]
"""
import argparse
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
synth = importlib.import_module("photometric-bundle-adjustment_amd.synth")
E = importlib.import_module("photometric-bundle-adjustment_amd.engine")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--texture", default="noise")
    ap.add_argument("--solve", action="store_true", help="time pba_solve (the device-steered LM loop) instead")
    ap.add_argument("--p21", action="store_true", help="the C5 pattern: the 21-px disk of radius √5 (bench.py DISK21)")
    args = ap.parse_args()
    import numpy as np
    import torch
    dev = torch.device("cuda", 0)
    pb, images = synth.c4_shard(dev, texture=args.texture)
    if args.p21:
        disk = np.array([(dx, dy) for dy in range(-2, 3) for dx in range(-2, 3) if dx * dx + dy * dy <= 5], np.float32)
        host = torch.from_numpy(pb.point_host.astype(np.int64)).to(dev)[:, None]
        uu = torch.from_numpy((pb.u_ref[:, 0][:, None] + disk[None, :, 0]).astype(np.int64)).to(dev)
        vv = torch.from_numpy((pb.u_ref[:, 1][:, None] + disk[None, :, 1]).astype(np.int64)).to(dev)
        pb.pattern = disk
        pb.host_intensity = images[host, vv, uu].float().cpu().numpy()
    eng = E.Engine(synth.PHOTOMETRIC, synth.PINHOLE, device=0, huber_width=9.0)
    eng.set_problem(pb, images_device_ptr=images.data_ptr())
    eng.set_fixed_frames(np.array([0, 1], np.int32))
    eng.set_state(pb.poses, pb.rho)
    eng.gn_linearize()
    if args.solve:
        eng.solve(max_iterations=2, function_tolerance=0.0)
        eng.set_state(pb.poses, pb.rho)
        s = eng.solve(max_iterations=args.iters, function_tolerance=0.0)
        print(f"{s['total_ms'] / max(s['iterations'], 1):.3f} ms per LM iteration (pba_solve), {s['successful_steps']} accepted, final cost {s['final_cost']!r}")
        eng.close()
        return
    t0 = time.perf_counter()
    for _ in range(args.iters):
        eng.gn_linearize()
        eng.gn_step(1e-4)
        eng.gn_candidate_cost()
    eng.synchronize()
    print(f"{1e3 * (time.perf_counter() - t0) / args.iters:.3f} ms per (linearise + step + candidate cost), host-synchronous")
    eng.close()


if __name__ == "__main__":
    main()
