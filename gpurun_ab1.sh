#!/bin/bash
# GPU: the distributed tests (incl. the two-process gloo solve) + a per-trial kernel trace of pba_solve at C4
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_distributed.py -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_dist.txt 2>&1 || { tail -30 gpurun_out/gpu_dist.txt; exit 1; }
tail -3 gpurun_out/gpu_dist.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gntrace -o run -- \
    python tools/gn_kernels.py --solve --iters 10 > gpurun_out/gntrace.log 2>&1 || { tail -5 gpurun_out/gntrace.log; exit 1; }
python3 tools/gn_trace.py gpurun_out/gntrace/run_kernel_trace.csv
