#!/bin/bash
# GPU box: config2_active parity + commit traces of two k_active_match trace builds
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; VARS=$2
mkdir -p $R/gpurun_out/$TAG
cd $R
for v in ${VARS//,/ }; do
  lib=$R/gf_orb_slam_amd/diag/libgfslam_${v}.so
  GF_LIB=$lib timeout -k 10 200 python -u -m pytest tests/test_pipeline_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread -k "config2_active" > gpurun_out/$TAG/$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(tail -1 gpurun_out/$TAG/$v.log)"
  case $rc in 0|1) ;; *) exit $rc;; esac
  case $v in *tr*) GF_LIB=$lib timeout -k 10 120 python -u scripts/am_trace.py gpurun_out/$TAG/$v.npz > gpurun_out/$TAG/$v.trace 2>&1 || exit $?; grep -v Warn gpurun_out/$TAG/$v.trace | grep -v amdgpu.ids;; esac
  case $v in *chk*) GF_LIB=$lib timeout -k 10 120 python -u scripts/am_check.py > gpurun_out/$TAG/$v.check 2>&1 || exit $?; grep -v amdgpu.ids gpurun_out/$TAG/$v.check;; esac
done
exit 0
