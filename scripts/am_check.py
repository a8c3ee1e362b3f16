"""Run the config2_active pipeline case (tests/test_pipeline_gpu.py) on a
GF_AM_CHECK build of k_active_match and print its commit checks: the RNG
history restarted from a saved batch against the step-by-step one, slot and
keypoint index ranges, the sigma^2 copy.
Usage: GF_LIB=gf_orb_slam_amd/diag/libgfslam_<variant>.so python scripts/am_check.py"""
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
buf = (ctypes.c_ulonglong * 80)()
lib().gf_debug_am_check(buf)
print("commits checked", buf[4], "rng restarts differing", buf[0], "slot out of range", buf[1],
      "claim out of range", buf[2], "sigma2 copies differing", buf[3])
if buf[0]:
    print("first: frame %d round %d T %d nb %d b %d sz %d npop %d pass %d" % tuple(
        ctypes.c_longlong(buf[i]).value for i in range(8, 16)))
    print("fast", [buf[16 + i] for i in range(31)])
    print("slow", [buf[48 + i] for i in range(31)])
