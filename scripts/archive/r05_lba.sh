#!/bin/bash
# GPU box: k_ba_solve variants — LBA parity (product), then per variant the
# config-4 timing table and the solve's phase stamps.
# Usage: scripts/r05_lba.sh TAG variant[,variant...]   (product = the in-tree library)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; VARS=$2
mkdir -p $R/gpurun_out/$TAG
cd $R
timeout -k 10 300 python -u -m pytest tests/test_lba_gpu.py tests/test_dropin_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/$TAG/pytest_lba.log 2>&1 || { tail -5 gpurun_out/$TAG/pytest_lba.log; exit 10; }
tail -1 gpurun_out/$TAG/pytest_lba.log
for v in ${VARS//,/ }; do
  case $v in product*) lib="";; *) lib=$R/gf_orb_slam_amd/diag/libgfslam_${v}.so;; esac
  GF_LIB=$lib timeout -k 10 120 python -u scripts/lba_timing.py > gpurun_out/$TAG/timing_$v.log 2>&1 || exit 11
  GF_LIB=$lib timeout -k 10 120 python -u scripts/lba_phases.py > gpurun_out/$TAG/phases_$v.log 2>&1 || exit 12
  echo "$v: $(grep 'B=1 ' gpurun_out/$TAG/timing_$v.log) | $(grep k_ba_solve gpurun_out/$TAG/timing_$v.log | head -1) | $(grep phases gpurun_out/$TAG/phases_$v.log)"
done
exit 0
