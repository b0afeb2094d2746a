#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/steps.txt
bash tools/gpu_steps.sh \
  600 gpurun_out/s8_tests.log python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_gn.py tests/test_gpu_pyramid.py tests/test_gpu_configs.py -k "large_patterns or pyramid or c5 or coarse or lm or reduced" -rf @@ \
  300 gpurun_out/s8_p21.log rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s8_p21 -o run -- python tools/gn_kernels.py --solve --iters 10 --p21 @@ \
  300 gpurun_out/s8_p8.log rocprofv3 --kernel-trace --output-format csv -d gpurun_out/s8_p8 -o run -- python tools/gn_kernels.py --solve --iters 10
cat gpurun_out/steps.txt
