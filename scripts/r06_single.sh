#!/bin/bash
# GPU box: one sequence alone (per-kernel HIP-event times, eager / graph) and
# the local-BA phase timing (scripts/lba_timing.py)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-single}
mkdir -p $R/gpurun_out/$TAG
cd $R
timeout -k 10 300 python scripts/single_prof.py 100 > gpurun_out/$TAG/single.json 2> gpurun_out/$TAG/single.err || exit 10
cat gpurun_out/$TAG/single.json
timeout -k 10 300 python scripts/lba_timing.py > gpurun_out/$TAG/lba.json 2> gpurun_out/$TAG/lba.err || exit 11
head -c 3000 gpurun_out/$TAG/lba.json
exit 0
