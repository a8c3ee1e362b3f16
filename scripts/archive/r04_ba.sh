#!/bin/bash
# GPU box: k_ba_solve workgroup size A/B (BA_SOLVE_THREADS 1024 / 512 / 256):
# solve phases, LBA wall time per window, and the LBA parity tests per build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for v in product ba512 ba256; do
  L=""; [ $v != product ] && L=$R/gf_orb_slam_amd/diag/libgfslam_$v.so
  GF_LIB=$L timeout -k 10 120 python scripts/lba_phases.py > gpurun_out/ba_phases_$v.log 2>&1 || exit 10
  GF_LIB=$L timeout -k 10 300 python scripts/lba_timing.py > gpurun_out/ba_timing_$v.log 2>&1 || exit 11
  echo "$v: $(grep phases gpurun_out/ba_phases_$v.log) | $(grep '^B=' gpurun_out/ba_timing_$v.log | tr '\n' ' ')"
done
for v in ba512 ba256; do
  GF_LIB=$R/gf_orb_slam_amd/diag/libgfslam_$v.so timeout -k 10 600 python -u -m pytest tests/test_lba_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ba_pytest_$v.log 2>&1 || exit 12
  tail -1 gpurun_out/ba_pytest_$v.log
done
