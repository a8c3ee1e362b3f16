"""Phase cycles of k_active_match (diagnostic build, `make stamp`): one
front end of B streams in the bench's GF regime (config 2: keyframe maps,
UpdateReference, 0.82 stale map descriptors; `fixed`: fixed maps, 0.93), stamps summed over frames and divided by frame-steps.
Usage: GF_LIB=gf_orb_slam_amd/diag/libgfslam_am.so python scripts/am_stamps.py [B] [steps] [fixed]"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from gf_orb_slam_amd import ORBextractor, scene  # noqa: E402
from gf_orb_slam_amd._lib import lib  # noqa: E402
from gf_orb_slam_amd.pipeline import FrontEnd  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
fixed = len(sys.argv) > 3 and sys.argv[3] == "fixed"  # else the bench regime: keyframe maps, UpdateReference
W = scene.Workload("euroc", B, n_scenes=32, period=32, seed=0, stale_desc=0.93 if fixed else 0.82)  # as bench.py
frames = W.render_all("cuda").contiguous()
ex = ORBextractor(1000, 1.2, 8, 1, 20)
M = 2000 if fixed else 2100
if fixed:
    maps = [(m[0], m[1]) for m in W.build_maps(lambda im: ex(im), M, device="cuda")]
else:
    maps = [(g["mp"], g["desc"], g["graph"]) for g in W.build_global_maps(lambda im: ex(im), M, device="cuda")]
fe = FrontEnd("euroc", 1000, B, M, 100)
for b in range(B):
    m = maps[W.scene_of[b]]
    fe.set_map(b, m[0], m[1])
    if len(m) > 2:
        fe.set_covis(b, m[2])
    fe.set_rng(b, 1 + b)
fe.set_source(frames, W.scene_of, W.phase)
T, V = W.boot_state()
fe.bootstrap(T, V, 0.0)
for _ in range(3):
    fe.step()
fe.sync()
f = lib().gf_debug_am_stamps
f.argtypes = [ctypes.c_void_p, ctypes.c_int]
st = np.zeros(24, np.uint64)
f(st.ctypes.data, 1)
fe.write("hist", np.zeros((B, 8), np.int32))
fe.prof_enable(True)
fe.prof_reset()
for _ in range(steps):
    fe.step()
fe.sync()
f(st.ctypes.data, 0)
prof = fe.prof_report()
h = fe.read("hist")
names = ["setup", "pool", "draws", "evals", "heap_pops", "commit_rng", "pool_update", "recount"]
per = st[:8].astype(np.float64) / (B * steps)
out = {"B": B, "steps": steps, "cycles_per_frame": {k: round(float(v)) for k, v in zip(names, per)},
       "logdets_per_frame": float(h[:, 6].sum()) / (B * steps), "matches_per_frame": float(h[:, 7].sum()) / (B * steps),
       "counts_per_frame": {k: round(float(st[i]) / (B * steps), 2) for i, k in
                            [(8, "draw_batches"), (9, "eval_calls"), (10, "evaluated"), (11, "rescans"),
                             (12, "rounds"), (13, "pops")]},
       "frame_cycles": {"max": int(st[16]), "mean": round(float(st[17]) / (B * steps))},
       "k_active_match_ms": prof["k_active_match"][0] / prof["k_active_match"][1],
       "k_onepoint_pre_ms": prof["k_onepoint_pre"][0] / prof["k_onepoint_pre"][1]}
print(json.dumps(out))
