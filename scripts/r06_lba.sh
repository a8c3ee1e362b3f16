#!/bin/bash
# GPU box: local-BA parity (tests/test_lba_gpu.py) on the product, then the
# per-kernel LBA timing (scripts/lba_timing.py) of the product and variants
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; VARS=$2
mkdir -p $R/gpurun_out/$TAG
cd $R
O=gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_lba_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 10; }
echo "lba tests: $(tail -1 $O/pytest.log)"
for v in ${VARS//,/ }; do
  case $v in product*) lib="";; *) lib=$R/gf_orb_slam_amd/diag/libgfslam_${v}.so;; esac
  GF_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_lba_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 12; }
  GF_LIB=$lib timeout -k 10 300 python scripts/lba_timing.py > $O/$v.txt 2> $O/$v.err || { tail -20 $O/$v.err; exit 11; }
  echo "== $v $(tail -1 $O/pytest_$v.log)"; grep -E "B=1 |k_ba_solve|B=64" $O/$v.txt | head -6
done
exit 0
