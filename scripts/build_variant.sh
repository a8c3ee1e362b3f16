# diagnostic library variant: build/var_$1/*.o with extra flags -> gf_orb_slam_amd/diag/libgfslam_$1.so
set -e
N=$1; shift
mkdir -p build/var_$N gf_orb_slam_amd/diag
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -Wall -Wno-unused-function"
for s in gf_orb_slam_amd/csrc/*.hip; do
  b=$(basename $s .hip); /opt/rocm/bin/hipcc $F "$@" -c $s -o build/var_$N/$b.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC build/var_$N/*.o build/*.cpp.o -L/opt/rocm/lib -lrccl -o gf_orb_slam_amd/diag/libgfslam_$N.so
