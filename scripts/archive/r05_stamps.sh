#!/bin/bash
# GPU box: k_active_match phase stamps (diagnostic build) at B = 1 and 256
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
mkdir -p $R/gpurun_out
cd $R
for B in 1 256; do
  GF_LIB=$R/gf_orb_slam_amd/diag/libgfslam_am.so timeout -k 10 300 python scripts/am_stamps.py $B 10 > gpurun_out/stamps_${TAG}_$B.json 2> gpurun_out/stamps_${TAG}_$B.err || exit 11
  cat gpurun_out/stamps_${TAG}_$B.json
done
