#!/bin/bash
# GPU box: one pipeline parity case on the product library and on diagnostic variants.
# Usage: scripts/r05_bisect.sh TAG "pytest -k expr" variant[,variant...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; K=$2; VARS=$3
mkdir -p $R/gpurun_out/$TAG
cd $R
for v in ${VARS//,/ }; do
  case $v in product*) lib="";; *) lib=$R/gf_orb_slam_amd/diag/libgfslam_${v}.so;; esac
  GF_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread -k "$K" > gpurun_out/$TAG/$v.log 2>&1
  echo "$v rc=$? $(tail -1 gpurun_out/$TAG/$v.log)"
done
exit 0
