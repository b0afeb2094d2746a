#!/usr/bin/env python3
"""Diagnostic: bench.py's C2 drop-in leg alone (real Ceres over include/pba_ceres.h, the CPU AutoDiff path and Ceres'
floor at C2 and on the 100k-block C4 sample), with the adapter's PrepareForEvaluation breakdown.  Not a parity check.
    python tools/probe/c2_probe.py"""
import importlib.util
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
B = importlib.util.module_from_spec(spec)
spec.loader.exec_module(B)


def main():
    import torch
    dev = torch.device("cuda", 0)
    full, images = B.synth.c4_shard(dev)
    out = B.c2_dropin(full, images.cpu().numpy(), B.host_cores()["usable"])
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    sys.exit(main())
