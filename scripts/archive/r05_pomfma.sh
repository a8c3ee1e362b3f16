#!/bin/bash
# GPU box: PoseOptimization with buildSystem on MFMA (PO_MFMA variant) against
# the oracle (pose / outlier parity) and the bench A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
mkdir -p $R/gpurun_out
cd $R
if [ "$2" != "ab-only" ]; then
GF_LIB=$R/gf_orb_slam_amd/diag/libgfslam_pomfma.so timeout -k 10 600 python -u -m pytest tests/test_pose_gpu.py "tests/test_pipeline_gpu.py::test_sequence_matches_oracle" tests/test_track_loss_gpu.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_pomfma_$TAG.log 2>&1
rc=$?
echo "variant pytest rc=$rc"; tail -3 gpurun_out/pytest_pomfma_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 12; fi
bash scripts/r05_ab.sh ab_$TAG pomfma,product || exit 11
fi
timeout -k 10 300 python scripts/pose_mfma_ab.py 400 80 > gpurun_out/pose_ab_product_$TAG.json || exit 13
GF_LIB=$R/gf_orb_slam_amd/diag/libgfslam_pomfma.so timeout -k 10 300 python scripts/pose_mfma_ab.py 400 80 > gpurun_out/pose_ab_pomfma_$TAG.json || exit 14
cat gpurun_out/pose_ab_*_$TAG.json
