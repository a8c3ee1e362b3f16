set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_dropin_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r03b_pytest.log 2>&1 || exit 10
bash scripts/r03_stamps.sh r03b || exit 11
