set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && rm -f gpurun_out/steps.txt
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_gn.py > gpurun_out/r6_gn_t30.log 2>&1 || exit 1
AB_ARGS="--no-c5 --no-c3 --no-live-traffic --no-shard-leg --gn-iterations 20" timeout -k 10 800 bash tools/ab_bench.sh base desc base desc > gpurun_out/ab_summary.log 2>&1
