# blur variants (diagnostic builds) + a tracking-priority check
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pipeline_gpu.py -k "priority or bench_shape" -m gpu -x -v --timeout 250 --timeout-method thread > gpurun_out/bx_pytest.log 2>&1 || exit 9
timeout -k 10 200 python scripts/kernel_times.py 512 5 > gpurun_out/bx0.json 2>/dev/null || exit 10
GF_LIB=gf_orb_slam_amd/diag/libgfslam_bx1.so timeout -k 10 200 python scripts/kernel_times.py 512 5 > gpurun_out/bx1.json 2>/dev/null || exit 11
GF_LIB=gf_orb_slam_amd/diag/libgfslam_bx2.so timeout -k 10 200 python scripts/kernel_times.py 512 5 > gpurun_out/bx2.json 2>/dev/null || exit 12
timeout -k 10 400 python bench.py --no-cpu-baseline --lba-batch 0 --pcie-steps 0 --single-stream-steps 0 > gpurun_out/bx_bench_prio.json 2> gpurun_out/bx_bench_prio.err || exit 13
timeout -k 10 400 python bench.py --no-cpu-baseline --lba-batch 0 --pcie-steps 0 --single-stream-steps 0 --no-track-priority > gpurun_out/bx_bench_noprio.json 2> gpurun_out/bx_bench_noprio.err || exit 14
