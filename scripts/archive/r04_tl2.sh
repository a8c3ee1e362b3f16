#!/bin/bash
# GPU box: the track-loss sequences, then the whole GPU suite and a short bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_track_loss_gpu.py -x -v -s --timeout 500 --timeout-method thread \
  -k "lost or miss" > gpurun_out/tl_chain.log 2>&1 || exit 11
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread \
  --deselect tests/test_track_loss_gpu.py > gpurun_out/pytest_tl.log 2>&1 || exit 12
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_tl.json 2> gpurun_out/bench_tl.err || exit 13
exit 0
