#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel trace and two PMC passes (FETCH_SIZE,
# WRITE_SIZE — separate passes as MI355X_MICROARCH.md prescribes).  Every GPU step has its own time limit;
# the script stops at the first crash/timeout (exit >= 2 or a signal).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-run}
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }

if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -q -rA ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3
  ok $rc || exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
  echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
  ok $rc || exit $rc
fi
timeout -k 10 600 python bench.py > gpurun_out/bench_${TAG}.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench_${TAG}.log
[ $rc -eq 0 ] || exit $rc
if [ -n "${EXTRA:-}" ]; then
  timeout -k 10 600 python $EXTRA > gpurun_out/extra_${TAG}.log 2>&1; rc=$?
  echo "extra rc=$rc"; tail -30 gpurun_out/extra_${TAG}.log
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_kt -o run -- \
      python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-c3 --no-live-traffic > gpurun_out/prof_${TAG}_kt.log 2>&1; rc=$?
  echo "rocprof kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $C --output-format csv -d gpurun_out/prof_${TAG}_$C -o run -- \
        python bench.py --steps 5 --warmup 2 --clock-warmup-s 0 --gn-iterations 2 --no-c3 --no-c5 --no-cpu-baseline --no-live-traffic > gpurun_out/prof_${TAG}_$C.log 2>&1; rc=$?
    echo "rocprof $C rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
fi
exit 0
