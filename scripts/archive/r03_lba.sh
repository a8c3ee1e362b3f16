# LBA: parity tests, per-window timing, k_ba_solve phases
set -o pipefail
mkdir -p gpurun_out
T=${1:-lba}
timeout -k 10 400 python -u -m pytest tests/test_lba_gpu.py tests/test_dropin_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit 10
timeout -k 10 200 python scripts/lba_timing.py > gpurun_out/${T}_timing.log 2>&1 || exit 11
timeout -k 10 200 python scripts/lba_phases.py > gpurun_out/${T}_phases.log 2>&1 || exit 12
