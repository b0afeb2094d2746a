set -u
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp && rm -f gpurun_out/steps.txt
timeout -k 10 700 bash tools/ab_bench.sh base prio base prio > gpurun_out/ab_summary.log 2>&1
