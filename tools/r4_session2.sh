#!/bin/bash
# Round-4 GPU session 2: distributed + GN tests after the export / import changes, the distributed trial trace, and the
# block-order FETCH A/B (tools/fetch_ab.sh).  Stops at the first crash / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/steps.txt
bash tools/gpu_steps.sh \
  600 gpurun_out/s2_tests.log python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
      tests/test_gpu_distributed.py tests/test_gpu_gn.py -rf @@ \
  300 gpurun_out/s2_dtrace.log rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s2_dtrace -o run -- \
      python tools/probe/dist_trace.py || exit $?
grep -q "rc=[^01]" gpurun_out/steps.txt && exit 3
bash tools/fetch_ab.sh
cat gpurun_out/steps.txt
