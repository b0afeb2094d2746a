#!/bin/bash
# One GPU round for the GN path (diagnostic): the GN parity tests, then a kernel trace of pba_solve at C4 (rendered
# images) summarised per trial (tools/gn_trace.py).  TESTS overrides the test selection; TAG names the outputs.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-gn}
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_gn.py} -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_tr -o run -- \
  python3 tools/gn_kernels.py --solve --iters 10 --texture render ${KARGS:-} > gpurun_out/${TAG}_k.log 2>&1 || exit 1
grep "per LM iteration" gpurun_out/${TAG}_k.log
python3 tools/gn_trace.py $(ls gpurun_out/${TAG}_tr/*kernel_trace.csv | head -1)
