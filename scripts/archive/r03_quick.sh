set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_pipeline_gpu.py tests/test_gf_gpu.py tests/test_lba_gpu.py tests/test_dropin_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03a_pytest.log 2>&1 || exit 10
timeout -k 10 400 python bench.py --no-cpu-baseline --lba-batch 0 --pcie-steps 0 > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err || exit 11
