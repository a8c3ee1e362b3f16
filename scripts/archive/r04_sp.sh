#!/bin/bash
# GPU box: single-sequence profile and active-match stamps, product vs $VARIANTS.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
T=${T:-sp}
timeout -k 10 300 python -u scripts/single_prof.py 100 > gpurun_out/${T}_single_product.json 2> gpurun_out/${T}_single_product.err || exit 11
for v in $VARIANTS; do
  GF_LIB=gf_orb_slam_amd/diag/libgfslam_$v.so timeout -k 10 300 python -u scripts/single_prof.py 100 > gpurun_out/${T}_single_$v.json 2> gpurun_out/${T}_single_$v.err || exit 12
done
GF_LIB=gf_orb_slam_amd/diag/libgfslam_am.so timeout -k 10 200 python scripts/am_stamps.py 1 30 > gpurun_out/${T}_am1.json 2> gpurun_out/${T}_am1.err || exit 13
exit 0
