#!/bin/bash
# GPU box: headline, single sequence and config 3 for the product and the
# library variants in $VARIANTS; then the single-sequence kernel profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
T=${T:-c3}
Q="--no-cpu-baseline --lba-batch 0 --pcie-steps 0 --budget-steps 0 --isolated-steps 0 --kernel-times events"
timeout -k 10 400 python bench.py $Q > gpurun_out/${T}_product.json 2> gpurun_out/${T}_product.err || exit 12
for v in $VARIANTS; do
  GF_LIB=gf_orb_slam_amd/diag/libgfslam_$v.so timeout -k 10 400 python bench.py $Q > gpurun_out/${T}_$v.json 2> gpurun_out/${T}_$v.err || exit 13
done
timeout -k 10 300 python -u scripts/single_prof.py 100 > gpurun_out/${T}_single.json 2> gpurun_out/${T}_single.err || exit 14
exit 0
