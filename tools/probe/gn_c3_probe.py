"""Diagnostic: the C3 Gauss-Newton problem alone (bench.py:gn_c3), for rocprofv3 kernel traces of one LM run."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import torch  # noqa: E402

if __name__ == "__main__":
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    torch.cuda.set_device(0)
    print(bench.gn_c3(iters, torch, 0, torch.device("cuda", 0)))
