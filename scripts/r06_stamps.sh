#!/bin/bash
# GPU box: k_active_match phase stamps and call counts (make stamp build) at B = 1 and 256
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-stamps}
mkdir -p $R/gpurun_out/$TAG
cd $R
for B in 1 256; do
  GF_LIB=$R/gf_orb_slam_amd/diag/libgfslam_am.so timeout -k 10 300 python scripts/am_stamps.py $B 5 > gpurun_out/$TAG/stamps_$B.json 2> gpurun_out/$TAG/stamps_$B.err || { tail -20 gpurun_out/$TAG/stamps_$B.err; exit 10; }
  cat gpurun_out/$TAG/stamps_$B.json
done
exit 0
