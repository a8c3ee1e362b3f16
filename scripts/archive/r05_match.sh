#!/bin/bash
# GPU box: matcher + pipeline parity, the group's PMC traffic, the bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-match}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_match_gpu.py tests/test_pipeline_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || exit 10
bash scripts/r05_pmc.sh pmc_$TAG || exit 12
bash scripts/r05_ab.sh $TAG product || exit 11
exit 0
