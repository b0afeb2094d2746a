#!/bin/bash
# Round-3 diagnostic call: counter passes (tools/r3_pmc.sh), a pba_solve kernel trace, the linearize A/B of two
# library variants (tools/ab_gn.sh) and the GN tests on the candidate variant.  Stops at the first crash/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_gn.sh ${AB_VARIANTS:-lin1 lin2} > gpurun_out/ab_lin.txt 2>&1; rc=$?; cat gpurun_out/ab_lin.txt; [ $rc -eq 0 ] || exit $rc
PBA_LIBRARY=$PWD/variants/libpba_${CAND:-lin2}.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    ${CAND_TESTS:-tests/test_gpu_gn.py tests/test_gpu_distributed.py} > gpurun_out/cand_tests.txt 2>&1; rc=$?
tail -3 gpurun_out/cand_tests.txt; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ "${PMC:-1}" = 1 ] || exit 0
bash tools/r3_pmc.sh > gpurun_out/r3_pmc.txt 2>&1; rc=$?; cat gpurun_out/r3_pmc.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/solve_kt -o run -- \
    python tools/gn_kernels.py --solve --iters 10 > gpurun_out/solve_kt.log 2>&1; rc=$?
python3 tools/gn_trace.py gpurun_out/solve_kt/run_kernel_trace.csv; exit $rc
