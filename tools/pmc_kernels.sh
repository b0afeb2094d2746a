#!/bin/bash
# Counter passes (diagnostic): the C5 21-px kernel (camera-table form), the GN linearisation and, for
# comparison, the headline block kernel; one rocprofv3 --pmc pass per counter group (tools/pmc_probe.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
SQ2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
SQ3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS"
ALL="$SQ1
$SQ2
$SQ3
FETCH_SIZE
WRITE_SIZE"
TAG=c5 KREGEX=photometric_block_kernel_multi ARGS="--steps 5 --warmup 2 --no-cpu-baseline --gn-iterations 0 --no-live-traffic" \
  GROUPS_LIST="$ALL" tools/pmc_probe.sh || exit $?
TAG=lin KREGEX=linearize_kernel SCRIPT=tools/gn_kernels.py ARGS="--iters 5" GROUPS_LIST="$ALL" tools/pmc_probe.sh || exit $?
TAG=blk KREGEX="photometric_block_kernel<" GROUPS_LIST="$SQ1
$SQ2
$SQ3" tools/pmc_probe.sh || exit $?
