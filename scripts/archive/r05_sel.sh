#!/bin/bash
# GPU box: a selection of GPU tests (args: pytest node ids / -k expressions after TAG)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_$TAG.log
exit $rc
