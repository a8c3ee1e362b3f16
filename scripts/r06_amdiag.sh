#!/bin/bash
# GPU box: config2_active parity on the product and the k_active_match
# diagnostic variants (AM_LSIG, GF_AM_CHECK, AM_SYNC_BAR), then the checks.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; VARS=$2
mkdir -p $R/gpurun_out/$TAG
cd $R
for v in ${VARS//,/ }; do
  case $v in product*) lib="";; *) lib=$R/gf_orb_slam_amd/diag/libgfslam_${v}.so;; esac
  GF_LIB=$lib timeout -k 10 200 python -u -m pytest tests/test_pipeline_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -k "config2_active" > gpurun_out/$TAG/$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(tail -1 gpurun_out/$TAG/$v.log)"
  case $rc in 0|1) ;; *) exit $rc;; esac
  case $v in *chk*) GF_LIB=$lib timeout -k 10 120 python -u scripts/am_check.py > gpurun_out/$TAG/$v.check 2>&1 || exit $?; cat gpurun_out/$TAG/$v.check | grep -v Warn;; esac
done
exit 0
