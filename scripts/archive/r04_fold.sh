#!/bin/bash
# GPU box: the track-loss tests, the whole GPU suite, the single-sequence
# per-kernel profile and a short bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_track_loss_gpu.py -x -v --timeout 500 --timeout-method thread \
  > gpurun_out/tl_all.log 2>&1 || exit 11
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread \
  --deselect tests/test_track_loss_gpu.py > gpurun_out/pytest_fold.log 2>&1 || exit 12
timeout -k 10 300 python -u scripts/single_prof.py 100 > gpurun_out/single_fold.json 2> gpurun_out/single_fold.err || exit 13
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --lba-batch 0 --config3-steps 0 \
  > gpurun_out/bench_fold.json 2> gpurun_out/bench_fold.err || exit 14
exit 0
