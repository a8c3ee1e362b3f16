#!/bin/bash
# GPU box: extraction alone (scripts/extract_times.py) under rocprofv3 kernel
# trace for library variants. Usage: scripts/r05_ext.sh TAG variant[,variant...] [B]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
VARS=$2
B=${3:-256}
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/$TAG
for v in ${VARS//,/ }; do
  case $v in product*) lib="";; *) lib=$R/gf_orb_slam_amd/diag/libgfslam_${v}.so;; esac
  rm -rf /tmp/ext_$v
  GF_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ext_$v -o run -- \
    python3 $R/scripts/extract_times.py $B 20 > $R/gpurun_out/$TAG/$v.log 2>&1 || exit 11
  f=$(find /tmp/ext_$v -name "run_kernel_stats.csv" | head -1)
  cp $f $R/gpurun_out/$TAG/${v}_kernel_stats.csv
  python3 - "$f" "$v" "$(grep extraction $R/gpurun_out/$TAG/$v.log)" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
print(sys.argv[2], sys.argv[3])
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print("   %-28s calls %5s avg %8.1f us" % (r["Name"][:28], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
  rm -rf /tmp/ext_$v
done
exit 0
