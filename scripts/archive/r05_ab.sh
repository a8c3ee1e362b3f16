#!/bin/bash
# GPU box: A/B of library variants on the bench (short legs).
# Usage: scripts/r05_ab.sh TAG variant[,variant...]   ("product" = gf_orb_slam_amd/libgfslam.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
VARS=$2
mkdir -p $R/gpurun_out/$TAG
cd $R
ARGS="--no-cpu-baseline --lba-batch 0 --config3-steps 0 --pcie-steps 0 --budget-steps 0 --isolated-steps 0 ${BENCH_ARGS}"
for v in ${VARS//,/ }; do
  lib=""
  case $v in product*) lib="";; *) lib=$R/gf_orb_slam_amd/diag/libgfslam_${v}.so;; esac
  GF_LIB=$lib timeout -k 10 300 python bench.py $ARGS --detail-out $R/gpurun_out/$TAG/detail_$v.json \
    > gpurun_out/$TAG/bench_$v.json 2> gpurun_out/$TAG/bench_$v.err || exit 11
  python3 - "$R/gpurun_out/$TAG/detail_$v.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = d.get("kernels", {})
pick = {n: k[n]["avg_ms"] for n in ("k_pyramid", "k_active_match", "k_blur_fast", "k_pose_opt_frames", "k_match_seq", "k_update_reference", "k_onepoint_pre", "k_select", "k_select_cells", "k_select_level", "k_fast_cells", "k_describe") if n in k}
print(sys.argv[2], "fps", d["value"], "single", d.get("single_stream", {}).get("ms_per_frame"), pick)
PY
done
exit 0
