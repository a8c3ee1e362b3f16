#!/bin/bash
# GPU box: headline A/B of the library variants in $VARIANTS (product before and after).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
T=${T:-abq}
Q="--no-cpu-baseline --lba-batch 0 --pcie-steps 0 --single-stream-steps 0 --budget-steps 0 --isolated-steps 0 --config3-steps 0 --kernel-times events"
timeout -k 10 300 python bench.py $Q > gpurun_out/${T}_product.json 2> gpurun_out/${T}_product.err || exit 12
for v in $VARIANTS; do
  GF_LIB=gf_orb_slam_amd/diag/libgfslam_$v.so timeout -k 10 300 python bench.py $Q > gpurun_out/${T}_$v.json 2> gpurun_out/${T}_$v.err || exit 13
done
timeout -k 10 300 python bench.py $Q > gpurun_out/${T}_product2.json 2> gpurun_out/${T}_product2.err || exit 14
exit 0
