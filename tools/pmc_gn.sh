#!/bin/bash
# Counter passes (diagnostic) over the kernels of one LM trial at C4 (rendered images, pba_solve): the linearisation,
# the λ-free elimination + decision, the assembly, the PCR levels and the update.  One rocprofv3 --pmc pass per group
# (tools/pmc_probe.sh); read with python tools/pmc_table.py gn.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
SQ2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
SQ3="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES"
TAG=${TAG:-gn} KREGEX="${KREGEX:-linearize_kernel|schur_free_decide|assemble_kernel|update_kernel|cr_level_wave|schur_gate}" \
  SCRIPT=tools/gn_kernels.py ARGS="--solve --iters 5 --texture render" GROUPS_LIST="$SQ1
$SQ2
$SQ3
FETCH_SIZE
WRITE_SIZE" tools/pmc_probe.sh
