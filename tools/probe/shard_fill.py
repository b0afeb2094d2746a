#!/usr/bin/env python3
"""Diagnostic: is the 1/8 shard's step set by workgroup imbalance over the CUs?  Times the headline
kernel on the first n blocks of the C4 problem's 1/8 host-keyframe shard for n around the shard's 50,120 blocks — 1536 and
1792 workgroups of 32 blocks are whole multiples of the 256 CUs, 1567 (the shard) leaves 31 CUs a seventh workgroup.

    python3 tools/probe/shard_fill.py
"""
import dataclasses
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
bench = importlib.import_module("bench")
synth = importlib.import_module("photometric-bundle-adjustment_amd.synth")
E = importlib.import_module("photometric-bundle-adjustment_amd.engine")
D = importlib.import_module("photometric-bundle-adjustment_amd.distributed")


def first_blocks(pb, n):
    keep = np.arange(n)
    return dataclasses.replace(pb, block_point=pb.block_point[keep], block_target=pb.block_target[keep],
                               u_obs=None if pb.u_obs is None else pb.u_obs[keep])


if __name__ == "__main__":
    import torch
    dev = torch.device("cuda", 0)
    full, images = synth.c4_shard(dev, n_frames=1000, n_points=100000, K=4)
    p8, _, _ = D.shard_problem(full, 8, 0)
    print(f"shard: {p8.n_blocks} blocks", flush=True)
    for n in (1280 * 32, 1536 * 32, 1552 * 32, p8.n_blocks, 1600 * 32, 1792 * 32, 2048 * 32):
        n = min(n, p8.n_blocks) if n > p8.n_blocks and n - p8.n_blocks < 32 else n
        pb = first_blocks(p8, n) if n <= p8.n_blocks else None
        if pb is None:  # more blocks than the shard: the 1/4 shard's first n
            p4, _, _ = D.shard_problem(full, 4, 0)
            pb = first_blocks(p4, n)
        eng = E.Engine(synth.PHOTOMETRIC, synth.PINHOLE, device=0, huber_width=9.0)
        eng.set_problem(pb, images_device_ptr=images.data_ptr())
        st = bench.make_states(pb, torch, dev, 7)
        el, k, _ = bench.time_evaluation(eng, st, 200, 20, 1.0, torch, None, dev)
        eng.close()
        print(f"{n:7d} blocks, {(n + 31) // 32:5d} workgroups: step {1e6 * el / 200:6.2f} us, kernel {k:6.2f} us, "
              f"{k / n * 1e3:.4f} ns per block", flush=True)
