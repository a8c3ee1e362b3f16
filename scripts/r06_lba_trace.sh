#!/bin/bash
# GPU box: rocprofv3 kernel trace of scripts/lba_timing.py at batch 1 (kernel
# durations and the gaps between them, without HIP events)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
mkdir -p $R/gpurun_out/$TAG
cd $R
export TMPDIR=/tmp
LBA_BATCHES=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/$TAG/prof -o run --output-format csv -- python3 scripts/lba_timing.py > $R/gpurun_out/$TAG/timing.txt 2>&1 || { tail -20 $R/gpurun_out/$TAG/timing.txt; exit 11; }
find $R/gpurun_out/$TAG/prof -name "*.csv" | head
exit 0
