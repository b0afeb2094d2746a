#!/usr/bin/env python3
"""Diagnostic: the multi-GPU LM loop's trial at C4 on ONE rank (pba_solve_distributed_comm over a one-rank RCCL
communicator, or an in-process group of --world engines sharing this GPU), for a rocprofv3 kernel trace whose
trial timeline (tools/gn_trace.py) splits into the replicated part (import, reduced solve, pose update, decision)
and the sharded part (Schur complement, export, point update, candidate linearisation).  Not a parity check.

    rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dt -o run -- python tools/probe/dist_trace.py
"""
import argparse
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
synth = importlib.import_module("photometric-bundle-adjustment_amd.synth")
E = importlib.import_module("photometric-bundle-adjustment_amd.engine")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=12)
    args = ap.parse_args()
    import numpy as np
    import torch
    pb, images = synth.c4_shard(torch.device("cuda", 0), texture="render")
    eng = E.Engine(synth.PHOTOMETRIC, synth.PINHOLE, device=0, huber_width=9.0)
    eng.set_problem(pb, images_device_ptr=images.data_ptr())
    eng.set_fixed_frames(np.array([0, 1], np.int32))
    eng.set_state(pb.poses, pb.rho)
    comm = E.Comm.rccl(E.Comm.unique_id(), 1, 0, 0)
    try:
        band = eng.gn_band()
        eng.solve_distributed_comm(band, comm, max_iterations=2)
        eng.set_state(pb.poses, pb.rho)
        s = eng.solve_distributed_comm(band, comm, max_iterations=args.iters, function_tolerance=0.0)
        print(f"{s['total_ms'] / max(s['iterations'], 1):.3f} ms per LM iteration (distributed loop, 1 rank), "
              f"{s['successful_steps']} accepted, final cost {s['final_cost']!r}")
        eng.set_state(pb.poses, pb.rho)
        s = eng.solve(max_iterations=args.iters, function_tolerance=0.0)
        print(f"{s['total_ms'] / max(s['iterations'], 1):.3f} ms per LM iteration (pba_solve), "
              f"{s['successful_steps']} accepted, final cost {s['final_cost']!r}")
    finally:
        comm.close()
        eng.close()


if __name__ == "__main__":
    main()
