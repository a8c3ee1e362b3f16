set -o pipefail
mkdir -p gpurun_out
GF_LIB=gf_orb_slam_amd/diag/libgfslam_am.so timeout -k 10 300 python scripts/am_stamps.py 512 5 > gpurun_out/${1:-am}_stamps.json 2> gpurun_out/${1:-am}_stamps.err
