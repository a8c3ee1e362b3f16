#!/bin/bash
# bench + rocprofv3 kernel-trace summary (run on the GPU box via gpurun)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python bench.py ${BENCH_ARGS} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 11
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline ${BENCH_ARGS} > $R/gpurun_out/bench_prof_$TAG.log 2>&1 || exit 12
exit 0
