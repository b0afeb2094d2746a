#!/bin/bash
# A/B the block kernel across prebuilt library variants (variants/libpba_<X>.so): one short bench per variant.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in "$@"; do
  PBA_LIBRARY=$PWD/variants/libpba_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline ${AB_ARGS:---gn-iterations 0} \
      > gpurun_out/ab_$v.log 2>&1 || { echo "variant $v failed"; tail -5 gpurun_out/ab_$v.log; exit 1; }
  tail -1 gpurun_out/ab_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value']/1e9,3), 'Gblk/s step', round(d['ms_per_step']*1e3,1), 'kernel', round(d['roofline']['kernel_avg_us'],1), 'gn', round(d['gn']['ms_per_iteration'],4) if d.get('gn') else None, d['gn']['breakdown_ms_per_iteration'] if d.get('gn') else None, 'c5_us', round(d['c5']['kernel_avg_us'],1) if d.get('c5') else None)"
done
