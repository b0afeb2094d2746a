#!/bin/bash
# GPU: solver tests after moving the LM record publish into the next trial's schur_kernel; per-trial trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")}"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_gn.py tests/test_gpu_pyramid.py tests/test_gpu_configs.py tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_gn.txt 2>&1 || { tail -30 gpurun_out/gpu_gn.txt; exit 1; }
tail -2 gpurun_out/gpu_gn.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gntrace -o run -- \
    python tools/gn_kernels.py --solve --iters 10 > gpurun_out/gntrace.log 2>&1 || { tail -5 gpurun_out/gntrace.log; exit 1; }
python3 tools/gn_trace.py gpurun_out/gntrace/run_kernel_trace.csv
timeout -k 10 200 python tools/gn_kernels.py --solve --iters 10
