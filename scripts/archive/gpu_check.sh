#!/bin/bash
# GPU box: parity tests, smoke, bench, rocprofv3 kernel-trace summary (run via gpurun).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || exit 10
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 13
timeout -k 10 500 python bench.py ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 11
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --single-stream-steps 0 --pcie-steps 0 --lba-batch 0 ${BENCH_ARGS} > $R/gpurun_out/bench_prof_$TAG.log 2>&1 || exit 12
exit 0
