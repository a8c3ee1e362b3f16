#!/bin/bash
# GPU box: bench A/B of the stream-group count (1024 sequences per GPU).
# Usage: scripts/r05_groups.sh TAG g[,g...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
cd $R
for g in ${2//,/ }; do
  BENCH_ARGS="--groups $g" bash scripts/r05_ab.sh $TAG/g$g product || exit 11
done
exit 0
