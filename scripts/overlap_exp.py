"""Experiment: B streams as G groups, each a FrontEnd with its own context
and HIP stream, stepped back to back so the groups' kernels overlap.
Usage: python scripts/overlap_exp.py B G [steps]"""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from gf_orb_slam_amd import synth  # noqa: E402
from gf_orb_slam_amd.pipeline import FrontEnd  # noqa: E402

B, G = int(sys.argv[1]), int(sys.argv[2])
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
graphs = len(sys.argv) > 4 and sys.argv[4] == "graph"
torch.cuda.set_device(0)
w, h = synth.CAMERAS["euroc"][:2]
fes = []
for g in range(G):
    fe = FrontEnd("euroc", 1000, B // G, 2000, gf_budget=100, seed=g)
    frames = np.stack([synth.synth_frame(w, h, synth.frame_seed(b, 0)) for b in range(8)])
    fe.load_frames(frames[np.arange(B // G) % 8])
    fe.build_maps()
    fes.append(fe)
for _ in range(3):
    for fe in fes:
        fe.step()
for fe in fes:
    fe.sync()
if graphs:
    for fe in fes:
        fe.capture_graph()
    for _ in range(2):
        for fe in fes:
            fe.step()
    for fe in fes:
        fe.sync()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    for fe in fes:
        fe.step()
for fe in fes:
    fe.sync()
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(f"B={B} G={G} graphs={graphs}: {B * steps / dt:.0f} fps, {dt / steps * 1e3:.3f} ms/step")
