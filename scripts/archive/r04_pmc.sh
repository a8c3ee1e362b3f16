#!/bin/bash
# GPU box: PMC passes of one 256-sequence front-end group alone (extraction
# LDS conflicts, HBM traffic per kernel) and of the LBA Schur product's
# matrix-core counters (config-4 windows, batches 1/8/64).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
bash scripts/pmc_extract.sh pmc_r04 || exit 11
python3 scripts/pmc_traffic.py gpurun_out/pmc_r04/summary.json gpurun_out/pmc_r04/traffic.json 256 \
  "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over scripts/kernel_times.py 256 3 (r04 build)" || exit 12
PASSES="SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT" \
  CMD="scripts/lba_timing.py" bash scripts/pmc_extract.sh pmc_lba_r04 || exit 13
exit 0
