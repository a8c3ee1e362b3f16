#!/bin/bash
# GPU box: active-matching parity on the product and the LDS-sigma^2 build, then bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; VARS=$2
mkdir -p $R/gpurun_out/$TAG
cd $R
O=gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_pipeline_gpu.py tests/test_gf_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "active or sequence or budget" > $O/pytest_product.log 2>&1 || { tail -30 $O/pytest_product.log; exit 10; }
echo "product: $(tail -1 $O/pytest_product.log)"
GF_LIB=$R/gf_orb_slam_amd/diag/libgfslam_lsig.so timeout -k 10 600 python -u -m pytest tests/test_pipeline_gpu.py tests/test_gf_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "active or sequence or budget" > $O/pytest_lsig.log 2>&1 || { tail -30 $O/pytest_lsig.log; exit 12; }
echo "lsig: $(tail -1 $O/pytest_lsig.log)"
exec_ab=1
bash scripts/r06_ab.sh $TAG $VARS
