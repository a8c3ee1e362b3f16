#!/bin/bash
# GPU box: full parity suite, smoke, bench (compact line + detail file), and
# the rocprofv3 kernel summary of the bench's timed configuration.
# Usage: scripts/r05_check.sh TAG [skip-tests]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05}
mkdir -p $R/gpurun_out
cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || exit 10
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 13
timeout -k 10 600 python bench.py ${BENCH_ARGS} --detail-out $R/gpurun_out/bench_detail_$TAG.json --kernel-trace-dir $R/gpurun_out/ktrace_$TAG > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 11
rm -f gpurun_out/ktrace_$TAG/*kernel_trace.csv
exit 0
