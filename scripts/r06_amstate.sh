#!/bin/bash
# GPU box: per-step state of config2_active on the product and on diagnostic builds
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; VARS=$2
mkdir -p $R/gpurun_out/$TAG
cd $R
for v in ${VARS//,/ }; do
  case $v in product*) lib="";; *) lib=$R/gf_orb_slam_amd/diag/libgfslam_${v}.so;; esac
  GF_LIB=$lib timeout -k 10 120 python -u scripts/am_state.py gpurun_out/$TAG/$v.npz > gpurun_out/$TAG/$v.state 2>&1 || exit $?
  echo "$v ok"
done
exit 0
