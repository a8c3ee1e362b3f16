#!/bin/bash
# GPU box: PMC passes (one per counter group) over a short bench run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-pmc}
B=${B:-256}
mkdir -p $R/gpurun_out/$TAG
export TMPDIR=/tmp
cd /tmp
ARGS="$R/bench.py --batch $B --groups 1 --steps 5 --warmup 2 --no-cpu-baseline --lba-batch 0 --single-stream-steps 0"
i=0
for CTRS in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" \
            "FETCH_SIZE" "WRITE_SIZE" ${EXTRA_PASSES}; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $CTRS -d $R/gpurun_out/$TAG/p$i -o run --output-format csv -- python3 $ARGS > $R/gpurun_out/$TAG/p$i.log 2>&1 || exit 20
done
exit 0
