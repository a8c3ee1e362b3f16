#!/bin/bash
# GPU box: full parity suite, the SEL_BUF_CELL=256 extraction variant, smoke,
# bench and the rocprofv3 kernel summary of the bench's timed configuration.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || exit 10
GF_LIB=$R/gf_orb_slam_amd/diag/libgfslam_c256.so timeout -k 10 200 python -u -m pytest tests/test_extract_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_c256_$TAG.log 2>&1 || exit 14
GF_LIB=$R/gf_orb_slam_amd/diag/libgfslam_am2p.so timeout -k 10 600 python -u -m pytest tests/test_gf_gpu.py tests/test_pipeline_gpu.py -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/pytest_am2p_$TAG.log 2>&1 || exit 15
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 13
timeout -k 10 600 python bench.py ${BENCH_ARGS} --kernel-trace-dir $R/gpurun_out/ktrace_$TAG > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 11
rm -f gpurun_out/ktrace_$TAG/*kernel_trace.csv  # (tens of MB; its timed-region table stays)
export TMPDIR=/tmp
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$TAG -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --single-stream-steps 0 --pcie-steps 0 --lba-batch 0 --config3-steps 0 ${BENCH_ARGS} > $R/gpurun_out/bench_prof_$TAG.log 2>&1 || exit 12
python3 $R/scripts/trace_timed.py $R/gpurun_out/prof_$TAG/run_kernel_trace.csv 5 20 4 > $R/gpurun_out/prof_$TAG/kernel_stats_timed.csv || exit 16
rm -f $R/gpurun_out/prof_$TAG/run_kernel_trace.csv
exit 0
