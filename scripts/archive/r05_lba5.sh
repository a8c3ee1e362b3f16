#!/bin/bash
# (historical: the BA_TRSV_NOFENCE / BA_TRAIL_PF / BA_TRAIL_RL variants this measured were
# removed from ba.hip after the measurement; results in profiles/r05/lba/)
# GPU box: pipelined trailing-update variant (BA_TRAIL_RL): parity, phase split, timing against the product.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out/lba5
D=$PWD/gf_orb_slam_amd/diag
GF_LIB=$D/libgfslam_rl.so timeout -k 10 300 python -u -m pytest tests/test_lba_gpu.py tests/test_dropin_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/lba5/rl_pytest.log 2>&1 || { tail -5 gpurun_out/lba5/rl_pytest.log; exit 5; }
tail -1 gpurun_out/lba5/rl_pytest.log
GF_LIB=$D/libgfslam_rlph.so timeout -k 10 120 python -u scripts/lba_chol_phases.py > gpurun_out/lba5/rlph.log 2>&1 || exit 6
GF_LIB=$D/libgfslam_chph.so timeout -k 10 120 python -u scripts/lba_chol_phases.py > gpurun_out/lba5/chph.log 2>&1 || exit 7
grep chol gpurun_out/lba5/rlph.log gpurun_out/lba5/chph.log
bash scripts/r05_lba.sh lba5b product,rl,product,rl
