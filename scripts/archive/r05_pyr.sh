#!/bin/bash
# GPU box: extraction parity (pyramid, blur, FAST, describe) then the short bench legs.
# Usage: scripts/r05_pyr.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pyr}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_extract_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || exit 10
bash scripts/r05_ab.sh $TAG product || exit 11
exit 0
