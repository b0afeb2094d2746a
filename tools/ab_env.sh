#!/bin/bash
# Per-kernel GN timings (rocprofv3 kernel trace of tools/gn_kernels.py) for values of one environment switch of the
# library (e.g. AB_VAR=PBA_CR_GJ tools/ab_env.sh wave split2 split3); each run has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  export "${AB_VAR}=$v"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/abe_$v -o run -- python tools/gn_kernels.py ${GN_ARGS:-} > gpurun_out/abe_$v.log 2>&1 \
      || { echo "variant $v failed"; tail -5 gpurun_out/abe_$v.log; exit 1; }
  echo "== $v: $(grep 'ms per' gpurun_out/abe_$v.log)"
  python3 tools/gn_trace.py gpurun_out/abe_$v/run_kernel_trace.csv || exit 1
done
