#!/bin/bash
# GPU box: rocprofv3 --pmc passes, one counter group per run (gfx950 slot
# limits: 8 SQ, 4 TCC — FETCH_SIZE takes 3, WRITE_SIZE 2 — so they get runs of
# their own). Default program: one 256-sequence front-end group alone
# (scripts/kernel_times.py). Summaries: python scripts/pmc_summary.py <dir>.
#   PASSES="A B C;D E" CMD="scripts/lba_timing.py" scripts/pmc_extract.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc}
PASSES=${PASSES:-"SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT;SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_SMEM GRBM_GUI_ACTIVE;FETCH_SIZE;WRITE_SIZE"}
CMD=${CMD:-"scripts/kernel_times.py 256 3"}
mkdir -p $R/gpurun_out/$TAG
export TMPDIR=/tmp
cd /tmp
IFS=';' read -ra PL <<< "$PASSES"
i=0
for CTRS in "${PL[@]}"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $CTRS -d /tmp/$TAG/p$i -o run --output-format csv -- python3 $R/$CMD > $R/gpurun_out/$TAG/p$i.log 2>&1 || exit 20
done
# raw per-dispatch CSVs stay on the box (tens of MB); the per-kernel averages come back
python3 $R/scripts/pmc_summary.py /tmp/$TAG > $R/gpurun_out/$TAG/summary.json || exit 21
exit 0
