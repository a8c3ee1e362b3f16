#!/bin/bash
# GPU box: the headline configuration with the per-kernel events on / off in
# the timed region and with 4 / 8 / 16 hardware queues.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
Q="--no-cpu-baseline --single-stream-steps 0 --lba-batch 0 --config3-steps 0 --pcie-steps 0 --budget-steps 0 --isolated-steps 0 --kernel-times events"
for cfg in "q4n:--no-prof-timed" "q8n:--no-prof-timed --hw-queues 8" "q16n:--no-prof-timed --hw-queues 16" "q8g8:--no-prof-timed --hw-queues 8 --groups 8" "q4n2:--no-prof-timed" "q8n2:--no-prof-timed --hw-queues 8"; do
  n=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 240 python bench.py $Q $a > gpurun_out/hwq_$n.json 2> gpurun_out/hwq_$n.err || exit 11
  python -c "import json;d=json.loads(open('gpurun_out/hwq_$n.json').readline());print('$n', d['value'], d['ms_per_step'], d['kernels']['k_match_project']['avg_ms'], d['kernels']['k_blur_fast']['avg_ms'])"
done
