#!/bin/bash
# A/B of a library variant: GN kernel trace (tools/ab_gn.sh), the C5 entry with and without the camera-table form, and
# the GN + pyramid GPU tests on the variant.  Each step has its own time limit; stops at the first crash/timeout.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
V=${V:-s4}
bash tools/ab_gn.sh $V || exit $?
PBA_LIBRARY=$PWD/variants/libpba_$V.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/solve_$V -o run -- \
    python tools/gn_kernels.py --solve --iters 10 > gpurun_out/solve_$V.log 2>&1 || { tail -5 gpurun_out/solve_$V.log; exit 1; }
grep "ms per" gpurun_out/solve_$V.log; python3 tools/gn_trace.py gpurun_out/solve_$V/run_kernel_trace.csv
for ct in ${C5_CT:-0 1}; do
  PBA_NO_CAM_TABLE=$ct PBA_LIBRARY=$PWD/variants/libpba_$V.so timeout -k 10 300 python bench.py --no-cpu-baseline --no-c2 \
      --no-c3 --gn-iterations 0 --steps 50 > gpurun_out/c5_${V}_nct$ct.log 2>&1 || { tail -5 gpurun_out/c5_${V}_nct$ct.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/c5_${V}_nct$ct.log').read().strip().splitlines()[-1]); print('no_cam_table=$ct', 'headline us', round(d['roofline']['kernel_avg_us'],2), 'c5', {k: d['c5'][k] for k in ('kernel_avg_us','ms_per_step')})"
done
PBA_LIBRARY=$PWD/variants/libpba_$V.so timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    ${TESTS:-tests/test_gpu_gn.py tests/test_gpu_pyramid.py tests/test_gpu_configs.py tests/test_gpu_distributed.py} > gpurun_out/tests_$V.txt 2>&1
rc=$?; tail -3 gpurun_out/tests_$V.txt; exit $rc
