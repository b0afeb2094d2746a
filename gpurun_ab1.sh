set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > gpurun_out/pytest_ab1.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_ab1.log
[ $rc -eq 0 ] || exit $rc
AB_ARGS="--gn-iterations 0 --no-c3 --no-c5" bash tools/ab_bench.sh base wg base wg || exit 1
AB_ARGS="--gn-iterations 10 --no-c5" bash tools/ab_bench.sh base wgpcr
