#!/bin/bash
# GPU box: (1) FETCH_SIZE calibration of scattered 4/32/64/128-B reads against a
# 16-B streaming read (scripts/exp/calib_fetch); (2) FETCH_SIZE, WRITE_SIZE and
# L2 hit/miss of one 256-sequence group alone (kernel_times.py), per kernel.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc_r05}
mkdir -p $R/gpurun_out/$TAG
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d /tmp/$TAG/calib/p1 -o run --output-format csv -- $R/scripts/exp/calib_fetch > $R/gpurun_out/$TAG/calib.log 2>&1 || exit 20
python3 $R/scripts/pmc_summary.py /tmp/$TAG/calib > $R/gpurun_out/$TAG/calib_summary.json || exit 21
cd $R
PASSES="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum" CMD="scripts/kernel_times.py 256 3" bash scripts/pmc_extract.sh $TAG/group || exit 22
exit 0
