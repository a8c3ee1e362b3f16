#!/bin/bash
# GPU box: PMC passes over scripts/lba_timing.py (batches 1, 8, 64 of config 4):
# the Schur product's matrix-core counters and k_ba_solve's LDS / wait counters.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
PASSES="SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT;SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE" \
  CMD="scripts/lba_timing.py" bash scripts/pmc_extract.sh pmc_lba_r05 || exit 13
exit 0
