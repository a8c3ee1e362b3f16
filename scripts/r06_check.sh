#!/bin/bash
# GPU box: full parity suite (product), the active-matching parity cases on the
# LDS-sigma^2 diagnostic build, smoke, bench (compact line + detail file with
# the rocprofv3 child's tables).
# Usage: scripts/r06_check.sh TAG [skip-tests]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06}
mkdir -p $R/gpurun_out/$TAG
cd $R
O=gpurun_out/$TAG
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 10
  echo "suite: $(tail -1 $O/pytest.log)"
  if [ -f gf_orb_slam_amd/diag/libgfslam_lsig.so ]; then
    GF_LIB=$R/gf_orb_slam_amd/diag/libgfslam_lsig.so timeout -k 10 600 python -u -m pytest tests/test_pipeline_gpu.py tests/test_gf_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -k "active or sequence or budget" > $O/pytest_lsig.log 2>&1 || exit 12
    echo "lsig: $(tail -1 $O/pytest_lsig.log)"
  fi
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 13
timeout -k 10 600 python bench.py ${BENCH_ARGS} --detail-out $R/$O/bench_detail.json --kernel-trace-dir $R/$O/ktrace --time-log $R/$O/time_log.txt > $O/bench.json 2> $O/bench.err || exit 11
rm -f $O/ktrace/*kernel_trace.csv
head -c 600 $O/bench.json
exit 0
