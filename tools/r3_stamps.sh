#!/bin/bash
# CR phase stamps (PBA_CR_STAMPS builds variants/libpba_crs<V>.so) of one trial per variant, then a GN kernel A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in ${STAMP_VARIANTS:-crs0 crs1}; do
  PBA_LIBRARY=$PWD/variants/libpba_$v.so timeout -k 10 300 python tools/gn_kernels.py --iters 1 > gpurun_out/stamps_$v.log 2>&1 || { tail -5 gpurun_out/stamps_$v.log; exit 1; }
  echo "== $v"; grep crstamp gpurun_out/stamps_$v.log | tail -40
done
bash tools/ab_gn.sh ${AB_VARIANTS:-cr1 s3}
