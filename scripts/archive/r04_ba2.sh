#!/bin/bash
# GPU box (historical: the look-ahead was measured and removed, see profiles/r04/ba/): k_ba_solve look-ahead (product) against the previous blocked LL^T
# (BA_LOOKAHEAD=0): LBA parity, solve phases and LBA wall time per window.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 600 python -u -m pytest tests/test_lba_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/ba2_pytest.log 2>&1 || exit 12
tail -1 gpurun_out/ba2_pytest.log
for v in product la0 product2; do
  L=""; [ $v == la0 ] && L=$R/gf_orb_slam_amd/diag/libgfslam_$v.so
  GF_LIB=$L timeout -k 10 120 python scripts/lba_phases.py > gpurun_out/ba2_phases_$v.log 2>&1 || exit 10
  GF_LIB=$L timeout -k 10 300 python scripts/lba_timing.py > gpurun_out/ba2_timing_$v.log 2>&1 || exit 11
  echo "$v: $(grep phases gpurun_out/ba2_phases_$v.log) | $(grep '^B=' gpurun_out/ba2_timing_$v.log | tr '\n' ' ')"
done
