#!/bin/bash
# GPU box: headline A/B of library variants (product first), then the
# active-match phase stamps at one stream and at a 256-stream group.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
Q="--no-cpu-baseline --lba-batch 0 --pcie-steps 0 --single-stream-steps 0 --budget-steps 0 --isolated-steps 0 --config3-steps 0 --kernel-times events"
T=${T:-ab4}
timeout -k 10 300 python bench.py $Q > gpurun_out/${T}_product.json 2> gpurun_out/${T}_product.err || exit 10
for v in $VARIANTS; do
  GF_LIB=gf_orb_slam_amd/diag/libgfslam_$v.so timeout -k 10 300 python bench.py $Q > gpurun_out/${T}_$v.json 2> gpurun_out/${T}_$v.err || exit 11
done
timeout -k 10 300 python bench.py $Q > gpurun_out/${T}_product2.json 2> gpurun_out/${T}_product2.err || exit 12
GF_LIB=gf_orb_slam_amd/diag/libgfslam_am.so timeout -k 10 200 python scripts/am_stamps.py 1 30 > gpurun_out/${T}_am1.json 2> gpurun_out/${T}_am1.err || exit 13
GF_LIB=gf_orb_slam_amd/diag/libgfslam_am.so timeout -k 10 200 python scripts/am_stamps.py 256 5 > gpurun_out/${T}_am256.json 2> gpurun_out/${T}_am256.err || exit 14
exit 0
