# (historical: the BA_TRSV_NOFENCE / BA_TRAIL_PF / BA_TRAIL_RL variants this measured were
# removed from ba.hip after the measurement; results in profiles/r05/lba/)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/lba3
GF_LIB=$PWD/gf_orb_slam_amd/diag/libgfslam_chph.so timeout -k 10 120 python -u scripts/lba_chol_phases.py > gpurun_out/lba3/chph.log 2>&1 || exit 5
GF_LIB=$PWD/gf_orb_slam_amd/diag/libgfslam_nofence.so timeout -k 10 300 python -u -m pytest tests/test_lba_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/lba3/nofence_pytest.log 2>&1 || exit 6
tail -1 gpurun_out/lba3/nofence_pytest.log
bash scripts/r05_lba.sh lba3b product,nofence,product,nofence
