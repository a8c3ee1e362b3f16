#!/bin/bash
# GPU box: bench A/B of the extraction gate's release stage (0 pyramid .. 4 describe; default 4)
# Usage: scripts/r05_gate.sh TAG stage[,stage...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
mkdir -p $R/gpurun_out/$TAG
cd $R
for st in ${2//,/ }; do
  BENCH_ARGS="--gate-stage $st" bash scripts/r05_ab.sh $TAG/g$st product || exit 11
done
exit 0
