#!/bin/bash
# GPU box: bench shape / gate A/B on the product library (short legs).
# Usage: scripts/r06_shape.sh TAG "name:args" ["name:args" ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
mkdir -p $R/gpurun_out/$TAG
cd $R
O=gpurun_out/$TAG
BASE="--no-cpu-baseline --lba-batch 0 --config3-steps 0 --budget-steps 0 --pcie-steps 0 --isolated-steps 0 --time-log-steps 0 --single-stream-steps 0 --kernel-times events"
for spec in "$@"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 400 python bench.py $BASE $args --detail-out $R/$O/$name.json > $O/$name.line 2> $O/$name.err || { tail -20 $O/$name.err; exit 11; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['config'].get('stream_groups'), d['config'].get('sequences_per_gpu'))" $O/$name.json "$name $args"
done
exit 0
