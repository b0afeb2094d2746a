#!/bin/bash
# SQ/GRBM counter passes over the bench's block kernel (one rocprofv3 --pmc pass per counter group, each
# under its own time limit; stops at the first failure).  Output: gpurun_out/pmc_<TAG>_<i>/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-probe}
ARGS=${ARGS:---steps 5 --warmup 2 --no-cpu-baseline --gn-iterations 0 --no-c5 --no-live-traffic}
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i + 1))
  timeout -s KILL 90 rocprofv3 --pmc $GROUP --kernel-include-regex "${KREGEX:-photometric_block_kernel}" \
      --output-format csv -d gpurun_out/pmc_${TAG}_$i -o run -- python ${SCRIPT:-bench.py} $ARGS > gpurun_out/pmc_${TAG}_$i.log 2>&1
  rc=$?; echo "pass $i ($GROUP) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<< "${GROUPS_LIST:-SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT}"
exit 0
