#!/bin/bash
# GPU box: single-sequence profile and active-match stamps, product (AM_CC 1) vs nocc (AM_CC 0).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
T=${T:-sp2}
timeout -k 10 300 python -u scripts/single_prof.py 100 > gpurun_out/${T}_single_product.json 2> gpurun_out/${T}_single_product.err || exit 11
GF_LIB=gf_orb_slam_amd/diag/libgfslam_nocc.so timeout -k 10 300 python -u scripts/single_prof.py 100 > gpurun_out/${T}_single_nocc.json 2> gpurun_out/${T}_single_nocc.err || exit 12
GF_LIB=gf_orb_slam_amd/diag/libgfslam_am.so timeout -k 10 200 python scripts/am_stamps.py 1 30 > gpurun_out/${T}_am1_cc.json 2> gpurun_out/${T}_am1_cc.err || exit 13
GF_LIB=gf_orb_slam_amd/diag/libgfslam_amnocc.so timeout -k 10 200 python scripts/am_stamps.py 1 30 > gpurun_out/${T}_am1_nocc.json 2> gpurun_out/${T}_am1_nocc.err || exit 14
exit 0
