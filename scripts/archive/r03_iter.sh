# GPU iteration: focused parity tests, active-match stamps, short bench (no CPU legs)
set -o pipefail
T=${1:-it}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gf_gpu.py tests/test_pipeline_gpu.py} -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit 10
bash scripts/r03_stamps.sh $T || exit 11
timeout -k 10 400 python bench.py --no-cpu-baseline --lba-batch 0 --pcie-steps 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 12
timeout -k 10 300 python scripts/kernel_times.py 512 5 > gpurun_out/${T}_ktimes.json 2> gpurun_out/${T}_ktimes.err || exit 13
