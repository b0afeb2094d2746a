#!/bin/bash
# pba_solve per-trial kernel traces of prebuilt library variants (variants/libpba_<X>.so), in the order given (repeat a
# name to interleave runs): tools/gn_kernels.py --solve under rocprofv3, summarised by tools/gn_trace.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i + 1))
  PBA_LIBRARY=$PWD/variants/libpba_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
      -d gpurun_out/abs_${v}_$i -o run -- python tools/gn_kernels.py --solve --iters 10 ${GN_ARGS:-} > gpurun_out/abs_${v}_$i.log 2>&1 \
      || { echo "variant $v failed"; tail -5 gpurun_out/abs_${v}_$i.log; exit 1; }
  echo "== $v ($i): $(grep 'ms per' gpurun_out/abs_${v}_$i.log)"
  python3 tools/gn_trace.py gpurun_out/abs_${v}_$i/run_kernel_trace.csv | grep -v cr_level || exit 1
done
