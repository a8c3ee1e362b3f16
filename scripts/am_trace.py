"""Run the config2_active pipeline case (tests/test_pipeline_gpu.py) for 12
steps on a GF_AM_TRACE build of k_active_match and save its per-commit
records (round, T, draws, pool size, committed RNG history, ...) of frames 0..7.
Usage: GF_LIB=gf_orb_slam_amd/diag/libgfslam_<variant>.so python scripts/am_trace.py OUT.npz"""
import ctypes
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))

import torch  # noqa: E402

from gf_orb_slam_amd._lib import lib  # noqa: E402
from test_pipeline_gpu import CASES, _setup  # noqa: E402

cam, nf, B, nmap, budget, gf, stale = CASES["config2_active"][:7]
W, frames, maps, fe, T, V = _setup(cam, nf, B, nmap, budget, gf, stale=stale)
counts = []
for _ in range(12):
    fe.step()
    torch.cuda.synchronize()
    cnt = np.zeros(8, np.uint32)
    tr = np.zeros((8, 2048, 48), np.uint32)
    lib().gf_debug_am_trace(tr.ctypes.data_as(ctypes.c_void_p), cnt.ctypes.data_as(ctypes.c_void_p))
    counts.append(cnt.copy())
np.savez_compressed(sys.argv[1], trace=tr, counts=np.array(counts))
print("commits per frame", cnt[:B], "per step", np.array(counts)[:, :B].tolist())
