#!/bin/bash
# GPU box: k_fast_cells with one wave per cell (FC_THREADS=64) against the
# product's four: extraction parity with the variant, the headline per build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
V=${V:-fc64}
timeout -k 10 300 python -u -m pytest tests/test_extract_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fc_pytest_product.log 2>&1 || exit 13
tail -1 gpurun_out/fc_pytest_product.log
GF_LIB=$R/gf_orb_slam_amd/diag/libgfslam_$V.so timeout -k 10 300 python -u -m pytest tests/test_extract_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/fc_pytest_$V.log 2>&1 || exit 12
tail -1 gpurun_out/fc_pytest_$V.log
Q="--no-cpu-baseline --single-stream-steps 0 --lba-batch 0 --config3-steps 0 --pcie-steps 0 --budget-steps 0 --isolated-steps 0"
for v in product $V product2 ${V}_2; do
  L=""; case $v in $V*) L=$R/gf_orb_slam_amd/diag/libgfslam_$V.so;; esac
  GF_LIB=$L timeout -k 10 300 python bench.py $Q > gpurun_out/fc_$v.json 2> gpurun_out/fc_$v.err || exit 11
  python -c "import json;d=json.loads(open('gpurun_out/fc_$v.json').readline());k=d['kernels'];print('$v', d['value'], d['ms_per_step'], {n:k[n]['avg_ms'] for n in ('k_fast_cells','k_blur_fast','k_select','k_describe') if n in k})"
done
