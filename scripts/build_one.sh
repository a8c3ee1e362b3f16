# diagnostic variant of one source: build/var_$1/<src>.o with extra flags, the rest from build/ -> gf_orb_slam_amd/diag/libgfslam_$1.so
# Usage: scripts/build_one.sh NAME SRC(e.g. gf) [flags...]
set -e
N=$1; S=$2; shift 2
mkdir -p build/var_$N gf_orb_slam_amd/diag
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-function"
/opt/rocm/bin/hipcc $F "$@" -c gf_orb_slam_amd/csrc/$S.hip -o build/var_$N/$S.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $(ls build/*.o | grep -v "build/$S.o") build/var_$N/$S.o -L/opt/rocm/lib -lrccl -o gf_orb_slam_amd/diag/libgfslam_$N.so
