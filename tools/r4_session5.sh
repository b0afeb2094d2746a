#!/bin/bash
# Round-4 GPU session 5: the 9-32 px tests with the 7-lanes-per-block C5 kernel, the C5 leg A/B (7 vs 8 lanes per block,
# interleaved), the one-rank nccl-group GN tests.  Stops at the first crash / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/steps.txt
B="python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-live-traffic --no-c3 --gn-iterations 0 --no-shard-leg"
bash tools/gpu_steps.sh \
  600 gpurun_out/s5_tests.log python -u -m pytest -q -s --timeout 300 --timeout-method thread -m gpu \
      tests/test_gpu_pyramid.py tests/test_gpu_parity.py tests/test_gpu_configs.py -k "pyramid or pattern or multi or c5" -rf @@ \
  300 gpurun_out/s5_ab_g7.log $B @@ \
  300 gpurun_out/s5_ab_g8.log env PBA_C5_LANES=8 $B @@ \
  300 gpurun_out/s5_ab_g7b.log $B @@ \
  300 gpurun_out/s5_ab_g8b.log env PBA_C5_LANES=8 $B @@ \
  400 gpurun_out/s5_nccl.log python -u -m pytest -q -s --timeout 300 --timeout-method thread -m gpu \
      tests/test_gpu_distributed.py -k "nccl_group or rccl_single" -rf
cat gpurun_out/steps.txt
