#!/bin/bash
# GPU box: bench A/B of library variants (product = in-tree libgfslam.so), short legs.
# Usage: scripts/r06_ab.sh TAG variant[,variant...] [pytest files to run first on the product]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; VARS=$2; TESTS=$3
mkdir -p $R/gpurun_out/$TAG
cd $R
O=gpurun_out/$TAG
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 10; }
  echo "tests: $(tail -1 $O/pytest.log)"
fi
ARGS="--no-cpu-baseline --lba-batch 0 --config3-steps 0 --budget-steps 0 --pcie-steps 0 --isolated-steps 0 --time-log-steps 0 ${BENCH_ARGS}"
for v in ${VARS//,/ }; do
  case $v in product*) lib="";; base*) lib=$R/gf_orb_slam_amd/diag/libgfslam_base.so;; *) lib=$R/gf_orb_slam_amd/diag/libgfslam_${v}.so;; esac
  GF_LIB=$lib timeout -k 10 400 python bench.py $ARGS --detail-out $R/$O/$v.json --kernel-trace-dir $R/$O/kt_$v > $O/$v.line 2> $O/$v.err || { tail -20 $O/$v.err; exit 11; }
  rm -f $O/kt_$v/*kernel_trace.csv
  python - "$O/$v.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); k = d["kernels"]
sel = ["k_active_match", "k_blur_fast", "k_match", "k_pose_opt_frames", "k_update_reference", "k_describe", "k_fe_gather", "k_onepoint_pre"]
print(sys.argv[2], d["value"], d["ms_per_step"], d.get("single_stream", {}).get("ms_per_frame"),
      {n: k[n]["avg_ms"] for n in sel if n in k})
PY
done
exit 0
