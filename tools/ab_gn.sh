#!/bin/bash
# Per-kernel GN timings (rocprofv3 kernel trace of tools/gn_kernels.py) for prebuilt library variants
# (variants/libpba_<X>.so); prints each variant's engine-kernel averages.  Each run has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  PBA_LIBRARY=$PWD/variants/libpba_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d gpurun_out/gnk_$v -o run -- python tools/gn_kernels.py ${GN_ARGS:-} > gpurun_out/gnk_$v.log 2>&1 \
      || { echo "variant $v failed"; tail -5 gpurun_out/gnk_$v.log; exit 1; }
  echo "== $v: $(grep 'ms per' gpurun_out/gnk_$v.log)"
  python3 - "$v" <<'PY'
import csv, sys
v = sys.argv[1]
for x in csv.DictReader(open(f"gpurun_out/gnk_{v}/run_kernel_stats.csv")):
    n = x["Name"]
    if "at::native" in n or "rocclr" in n or "tile_images" in n:
        continue
    print(f"  {n[:64]:64s} {x['Calls']:>4s} {float(x['AverageNs']) / 1e3:8.2f} us")
PY
done
