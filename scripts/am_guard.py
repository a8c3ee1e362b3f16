"""Run the config2_active pipeline case (tests/test_pipeline_gpu.py) on a
GF_AM_GUARD build and report k_active_match's LDS sentinel check.
Usage: GF_LIB=gf_orb_slam_amd/diag/libgfslam_guard.so python scripts/am_guard.py"""
import ctypes
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))

import torch  # noqa: E402

from gf_orb_slam_amd._lib import lib  # noqa: E402
from test_pipeline_gpu import CASES, _setup  # noqa: E402

cam, nf, B, nmap, budget, gf, stale = CASES["config2_active"][:7]
W, frames, maps, fe, T, V = _setup(cam, nf, B, nmap, budget, gf, stale=stale)
for _ in range(12):
    fe.step()
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 2)()
lib().gf_debug_am_guard(buf)
print("guard: corrupted sentinel dwords", buf[0], "frames checked", buf[1])
