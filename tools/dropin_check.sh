#!/bin/bash
# The Ceres drop-in on the GPU: its parity tests (C1/C2 drop-in, EUCM + bicubic against PhotometricError<8>, the
# callback protocol), then tools/probe/c2_probe.py twice (C2 and the C4 sample against CPU AutoDiff and Ceres' floor).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -f gpurun_out/steps.txt
bash tools/gpu_steps.sh \
  600 gpurun_out/s6_tests.log python -u -m pytest -q -s --timeout 300 --timeout-method thread -m gpu \
      tests/test_gpu_configs.py tests/test_gpu_bicubic.py tests/test_gpu_parity.py -k "dropin or ceres or adapter or callback" -rf @@ \
  600 gpurun_out/s6_c2a.log python tools/probe/c2_probe.py @@ \
  600 gpurun_out/s6_c2b.log python tools/probe/c2_probe.py
cat gpurun_out/steps.txt
