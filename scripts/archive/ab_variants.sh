# bench (headline legs only) with diagnostic library variants: product, then each GF_LIB
set -o pipefail
mkdir -p gpurun_out
Q="--no-cpu-baseline --lba-batch 0 --pcie-steps 0 --single-stream-steps 0 --budget-steps 0 --isolated-steps 0"
T=${1:-ab}; shift
timeout -k 10 300 python bench.py $Q > gpurun_out/${T}_product.json 2> gpurun_out/${T}_product.err || exit 10
for v in "$@"; do
  GF_LIB=gf_orb_slam_amd/diag/libgfslam_$v.so timeout -k 10 300 python bench.py $Q > gpurun_out/${T}_$v.json 2> gpurun_out/${T}_$v.err || exit 11
done
