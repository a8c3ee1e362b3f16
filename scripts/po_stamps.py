"""Diagnostic: phase cycles of k_pose_opt from a GF_PO_STAMP build of the
library (build_exp/libgfslam_postamp.so copied over gf_orb_slam_amd/ on the box).
Usage: python scripts/am_stamps.py [B] [steps]"""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from gf_orb_slam_amd import synth, _lib  # noqa: E402
from gf_orb_slam_amd.pipeline import FrontEnd  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
torch.cuda.set_device(0)
w, h = synth.CAMERAS["euroc"][:2]
fe = FrontEnd("euroc", 1000, B, 2000, gf_budget=100, seed=0)
frames = np.stack([synth.synth_frame(w, h, synth.frame_seed(b, 0)) for b in range(min(B, 8))])
fe.load_frames(frames[np.arange(B) % len(frames)])
fe.build_maps()
for _ in range(3):
    fe.step()
fe.sync()
lib = _lib.lib()
fn = lib.gf_debug_po_stamps
fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
buf = (ctypes.c_ulonglong * 8)()
fn(buf, 1)
for _ in range(steps):
    fe.step()
fe.sync()
fn(buf, 1)
names = ["(other)", "pass build", "ldlt+exp", "pass eval", "decide", "outliers", "-", "-"]
tot = sum(buf[i] for i in range(6))
per = B * steps
print(f"cycles per frame (B={B}, steps={steps}): total {tot / per:.0f}")
for i, nme in enumerate(names):  # (logdet) is inside eval0 + heaploop
    print(f"  {nme:12s} {buf[i] / per:10.0f}  {100.0 * buf[i] / max(tot, 1):5.1f}%")
print("matched per frame", fe.n_active.float().mean().item())
