#!/bin/bash
# Round-4 GPU session 3: GN / pyramid / configs tests, then the full bench line.  Stops at the first crash / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/steps.txt
bash tools/gpu_steps.sh \
  900 gpurun_out/s3_tests.log python -u -m pytest -q -s --timeout 600 --timeout-method thread -m gpu \
      tests/test_gpu_gn.py tests/test_gpu_pyramid.py tests/test_gpu_configs.py tests/test_gpu_parity.py -rf @@ \
  600 gpurun_out/bench_${TAG:-s3}.log python bench.py
cat gpurun_out/steps.txt
