#!/bin/bash
# GPU box: host launch order of the gated stream groups (bench --enqueue
# step | split | ring), the headline rate and the extraction-gate hand-over gaps from
# the rocprof child's kernel trace (scripts/gate_gaps.py).
set -o pipefail
timeout -k 10 60 ./scripts/exp/gate_probe > gpurun_out/gate_probe.log 2>&1; echo probe rc $?
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
Q="--no-cpu-baseline --single-stream-steps 0 --lba-batch 0 --config3-steps 0 --pcie-steps 0 --budget-steps 0 --isolated-steps 0"
for cfg in "step:--enqueue step" "ring:--enqueue ring" "split:--enqueue split" "step2:--enqueue step" "ring2:--enqueue ring"; do
  n=${cfg%%:*}; a=${cfg#*:}
  timeout -k 10 300 python bench.py $Q $a --kernel-trace-dir gpurun_out/enq_$n > gpurun_out/enq_$n.json 2> gpurun_out/enq_$n.err || exit 11
  python -c "import json;d=json.loads(open('gpurun_out/enq_$n.json').readline());print('$n', d['value'], d['ms_per_step'], d['host_enqueue'])"
  python scripts/gate_gaps.py gpurun_out/enq_$n/run_kernel_trace.csv | tee gpurun_out/enq_${n}_gaps.json
  rm -f gpurun_out/enq_$n/run_kernel_trace.csv
done
