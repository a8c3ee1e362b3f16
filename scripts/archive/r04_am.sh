#!/bin/bash
# GPU box: the GPU suite; the active-matching and front-end parity tests on a
# build with a 96-entry candidate capacity (most frames take the overflow
# pass); the headline A/B against the full-capacity build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread \
  > gpurun_out/pytest_am.log 2>&1 || exit 11
GF_LIB=$R/gf_orb_slam_amd/diag/libgfslam_amcc96.so timeout -k 10 600 python -u -m pytest tests/test_gf_gpu.py \
  tests/test_pipeline_gpu.py -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/pytest_amcc96.log 2>&1 || exit 12
VARIANTS=amccfull T=ab10 bash scripts/r04_abq.sh || exit 13
exit 0
