#!/bin/bash
# GPU box: the GPU suite, single-sequence profiles (product vs one-wave pose
# LM), LBA parity + timing, a short bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 500 --timeout-method thread \
  > gpurun_out/pytest_c.log 2>&1 || exit 11
timeout -k 10 300 python -u scripts/single_prof.py 100 > gpurun_out/single_c.json 2> gpurun_out/single_c.err || exit 12
GF_LIB=gf_orb_slam_amd/diag/libgfslam_nowide.so timeout -k 10 300 python -u scripts/single_prof.py 100 \
  > gpurun_out/single_c_nowide.json 2> gpurun_out/single_c_nowide.err || exit 13
timeout -k 10 200 python scripts/lba_timing.py > gpurun_out/lba_c_timing.log 2>&1 || exit 14
timeout -k 10 200 python scripts/lba_phases.py > gpurun_out/lba_c_phases.log 2>&1 || exit 15
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --lba-batch 0 --config3-steps 0 \
  > gpurun_out/bench_c.json 2> gpurun_out/bench_c.err || exit 16
exit 0
