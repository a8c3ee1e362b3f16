"""Run the config2_active pipeline case (tests/test_pipeline_gpu.py) for 12
steps and save each step's RNG state, stage counters and claims, so that two
builds of k_active_match can be compared step by step without instrumenting
the kernel. Usage: [GF_LIB=...] python scripts/am_state.py OUT.npz"""
import os
import sys

import numpy as np

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "tests"))

import torch  # noqa: E402

from test_pipeline_gpu import CASES, _setup  # noqa: E402

cam, nf, B, nmap, budget, gf, stale = CASES["config2_active"][:7]
W, frames, maps, fe, T, V = _setup(cam, nf, B, nmap, budget, gf, stale=stale)
out = {k: [] for k in ("rng", "stats", "kp2mp", "left", "base")}
for _ in range(12):
    fe.step()
    torch.cuda.synchronize()
    for k in out:
        out[k].append(fe.read(k).copy())
np.savez_compressed(sys.argv[1], **{k: np.array(v) for k, v in out.items()})
print("saved", sys.argv[1])
