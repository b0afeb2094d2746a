#!/usr/bin/env python3
"""Diagnostic (not a test): pba_solve on the whole C4 problem against pba_solve_distributed_comm over an in-process group
of W shard engines on one GPU, after 1, 2 and 4 LM iterations — max pose / relative inverse-distance differences and
the cost difference, for W = 1 (same sums, other code path) and W = 8."""
import importlib
import os
import sys
import threading

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
synth = importlib.import_module("photometric-bundle-adjustment_amd.synth")
E = importlib.import_module("photometric-bundle-adjustment_amd.engine")
D = importlib.import_module("photometric-bundle-adjustment_amd.distributed")


def main():
    import torch
    pb, images = synth.c4_shard(torch.device("cuda", 0), texture="render")

    def mk(p):
        e = E.Engine(0, 0, huber_width=9.0)
        e.set_problem(p, images_device_ptr=images.data_ptr())
        e.set_fixed_frames(np.array([0, 1], np.int32))
        e.set_state(p.poses, p.rho)
        return e

    full = mk(pb)
    for world in (1, 8):
        sh = []
        for r in range(world):
            sub, pids, _ = D.shard_problem(pb, world, r)
            sh.append((mk(sub), pids))
        comms = E.Comm.local_group(world)
        band = max(e.gn_band() for e, _ in sh)
        for iters in (1, 2, 4):
            full.set_state(pb.poses, pb.rho)
            ref = full.solve(max_iterations=iters)
            pr, rr = full.get_state()
            for e, pids in sh:
                e.set_state(pb.poses, pb.rho[pids])
            res = [None] * world
            th = [threading.Thread(target=lambda r=r: res.__setitem__(r, sh[r][0].solve_distributed_comm(
                band, comms[r], max_iterations=iters))) for r in range(world)]
            [t.start() for t in th]
            [t.join() for t in th]
            p0, _ = sh[0][0].get_state()
            rho = np.zeros(pb.n_points)
            for e, pids in sh:
                rho[pids] = e.get_state()[1]
            dpose = np.abs(p0 - pr).max()
            step = np.abs(pr - pb.poses).max()
            print(f"W={world} iters={iters}: {res[0]['successful_steps']}/{ref['successful_steps']} accepted, cost "
                  f"{abs(res[0]['final_cost'] - ref['final_cost']) / ref['final_cost']:.2e} rel, max|Δpose| {dpose:.3e} "
                  f"(max pose change {step:.3e}), max rel Δρ {np.abs(rho - rr).max() / np.abs(rr).max():.3e}", flush=True)
        for c in comms:
            c.close()
        for e, _ in sh:
            e.close()
    full.close()


if __name__ == "__main__":
    main()
