#!/bin/bash
# GPU box: bench shapes (sequences / stream groups) on the current build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
Q="--no-cpu-baseline --lba-batch 0 --pcie-steps 0 --single-stream-steps 0 --budget-steps 0 --isolated-steps 0 --config3-steps 0 --kernel-times events"
SHAPES=${SHAPES:-1024:4 768:3 1280:5 1536:6 2048:8 1024:2}
for sh in $SHAPES; do
  b=${sh%%:*}; g=${sh#*:}
  timeout -k 10 300 python bench.py $Q --batch $b --groups $g > gpurun_out/shape_${b}_${g}.json 2> gpurun_out/shape_${b}_${g}.err || exit 11
  python -c "import json;d=json.loads(open('gpurun_out/shape_${b}_${g}.json').readline());print('$b/$g', d['value'], d['ms_per_step'])"
done
exit 0
