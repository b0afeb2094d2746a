#!/bin/bash
# Round-4 GPU session 4: the pyramid / 9-32 px tests (the flat-row C5 kernel), then the C5 leg A/B (flat rows vs 8 lanes
# per block, interleaved) through bench.py's c5 entry.  Stops at the first crash / timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/steps.txt
bash tools/gpu_steps.sh \
  600 gpurun_out/s4_tests.log python -u -m pytest -q -s --timeout 300 --timeout-method thread -m gpu \
      tests/test_gpu_pyramid.py tests/test_gpu_parity.py tests/test_gpu_configs.py -k "pyramid or pattern or multi or c5 or read_back" -rf @@ \
  400 gpurun_out/s4_lmstate.log python -u -m pytest -q -s --timeout 300 --timeout-method thread -m gpu \
      tests/test_gpu_configs.py tests/test_gpu_gn.py -k "c1_engine_lm_matches or c3_engine_lm" -rf @@ \
  300 gpurun_out/s4_ab_flat1.log python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-live-traffic --no-c3 --gn-iterations 0 --no-shard-leg @@ \
  300 gpurun_out/s4_ab_flat0.log env PBA_FLAT_ROWS=0 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-live-traffic --no-c3 --gn-iterations 0 --no-shard-leg @@ \
  300 gpurun_out/s4_ab_flat1b.log python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-live-traffic --no-c3 --gn-iterations 0 --no-shard-leg @@ \
  300 gpurun_out/s4_ab_flat0b.log env PBA_FLAT_ROWS=0 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-live-traffic --no-c3 --gn-iterations 0 --no-shard-leg @@ \
  600 gpurun_out/c2_probe_4096.log python tools/probe/c2_probe.py
cat gpurun_out/steps.txt
