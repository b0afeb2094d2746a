#!/usr/bin/env python3
"""Diagnostic (host side): the fixed cost of the bench's timed region.  At the driver's K = 20 the
1/8 shard's step was 10.07 µs for an 8.43-µs kernel: ≈ 33 µs per run outside the kernels.  This times the same region
(barrier-free, one GPU) with three completion forms, R repetitions each, interleaved:

  blocking — hipStreamSynchronize on the engine stream, then torch.cuda.synchronize() (round 5's region);
  polled   — pba_synchronize (a marker event polled, then the stream synchronisation), then torch.cuda.synchronize();
  device   — torch.cuda.synchronize() alone;

and reports per form the median step (host wall ÷ K), the events' kernel time per step, and their difference × K (the
fixed cost).  Also the start latency: host time from t0 to the first launch's enqueue return.

    python3 tools/probe/sync_probe.py [--steps 20] [--reps 15]
"""
import argparse
import importlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
bench = importlib.import_module("bench")
synth = importlib.import_module("photometric-bundle-adjustment_amd.synth")
E = importlib.import_module("photometric-bundle-adjustment_amd.engine")
D = importlib.import_module("photometric-bundle-adjustment_amd.distributed")


def region(eng, states, steps, form, torch, dev):
    stream = torch.cuda.ExternalStream(eng.stream(), device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    pp = [states[i & 1][0].data_ptr() for i in range(steps)]
    rr = [states[i & 1][1].data_ptr() for i in range(steps)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    eng.evaluate_states_device(pp, rr, True, sync=False)
    t_enq = time.perf_counter() - t0
    e1.record(stream)
    if form == "blocking":
        stream.synchronize()
        torch.cuda.synchronize()
    elif form == "polled":
        eng.synchronize()
        torch.cuda.synchronize()
    else:
        torch.cuda.synchronize()
    t1 = time.perf_counter()
    return (t1 - t0) / steps * 1e6, e0.elapsed_time(e1) * 1e3 / steps, t_enq * 1e6


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=15)
    args = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    full, images = synth.c4_shard(dev, n_frames=1000, n_points=100000, K=4)
    for name, pb in (("shard 1/8", D.shard_problem(full, 8, 0)[0]), ("full C4", full)):
        eng = E.Engine(synth.PHOTOMETRIC, synth.PINHOLE, device=0, huber_width=9.0)
        eng.set_problem(pb, images_device_ptr=images.data_ptr())
        st = bench.make_states(pb, torch, dev, 7)
        bench.time_evaluation(eng, st, args.steps, 5, 0.3, torch, None, dev)  # clocks up, warm
        res = {f: [] for f in ("blocking", "polled", "device")}
        for _ in range(args.reps):
            for f in res:
                res[f].append(region(eng, st, args.steps, f, torch, dev))
        eng.close()
        print(f"{name}: {pb.n_blocks} blocks, K = {args.steps}", flush=True)
        for f, v in res.items():
            a = np.array(v)
            step, kern, enq = np.median(a[:, 0]), np.median(a[:, 1]), np.median(a[:, 2])
            print(f"  {f:8s} step {step:7.2f} us (min {a[:, 0].min():7.2f})  kernel {kern:6.2f} us  "
                  f"fixed {(step - kern) * args.steps:6.1f} us per run  enqueue {enq / args.steps:5.2f} us per step",
                  flush=True)
