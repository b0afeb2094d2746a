#!/bin/bash
# FETCH_SIZE / WRITE_SIZE / kernel time of the headline launch for two block orders of the same C4 problem
# (bench.py --traffic-probe --block-order point|morton), interleaved; one rocprofv3 pass per counter, each under its
# own time limit (tools/gpu_steps.sh).  Output: gpurun_out/fab_<order>_<ctr>_<i>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
K='photometric_block_kernel<0, 8, 1, float>'
args=()
for i in 1 2; do
  for o in point morton; do
    for c in FETCH_SIZE WRITE_SIZE; do
      args+=(120 gpurun_out/fab_${o}_${c}_$i.log rocprofv3 --pmc $c --kernel-include-regex "$K" --output-format csv \
             -d gpurun_out/fab_${o}_${c}_$i -o run -- python bench.py --traffic-probe --block-order $o @@)
    done
    args+=(120 gpurun_out/fab_${o}_kt_$i.log rocprofv3 --kernel-trace --stats --output-format csv \
           -d gpurun_out/fab_${o}_kt_$i -o run -- python bench.py --traffic-probe --block-order $o @@)
  done
done
unset 'args[${#args[@]}-1]'
bash tools/gpu_steps.sh "${args[@]}"
