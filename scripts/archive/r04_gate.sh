#!/bin/bash
# GPU box: headline with the extraction gate released after each stage.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
Q="--no-cpu-baseline --lba-batch 0 --pcie-steps 0 --single-stream-steps 0 --budget-steps 0 --isolated-steps 0 --config3-steps 0 --kernel-times events"
for st in ${STAGES:-4 3 2 4}; do
  timeout -k 10 300 python bench.py $Q --gate-stage $st > gpurun_out/gate_$st.json 2> gpurun_out/gate_$st.err || exit 11
  python -c "import json;d=json.loads(open('gpurun_out/gate_$st.json').readline());print('stage $st', d['value'], d['ms_per_step'])"
done
exit 0
