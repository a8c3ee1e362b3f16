#!/bin/bash
# GPU box: per-kernel PMC of one 256-sequence group alone on this round's build
# (scripts/kernel_times.py, the bench's distinct-frame workload): FETCH_SIZE,
# WRITE_SIZE (HBM traffic, gfx950 corrections in scripts/pmc_traffic.py), and
# the VALU / LDS / wave counters. One counter group per rocprofv3 run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc_r06}
cd $R
PASSES="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_SALU;GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" CMD="scripts/kernel_times.py 256 3" bash scripts/pmc_extract.sh $TAG || exit $?
python3 scripts/pmc_traffic.py gpurun_out/$TAG/summary.json gpurun_out/$TAG/pmc_traffic.json 256 "profiles/r06/$TAG (scripts/r06_pmc.sh, one 256-sequence group alone, r06 build)" || exit 23
exit 0
