"""Per-kernel device time of one front-end group alone (no overlapping
groups): B sequences of the bench workload, HIP events per launch.
Usage: python scripts/kernel_times.py [B] [steps] [stale] [fixed]  (stale
map-descriptor fraction, default 0.82 with keyframe maps + UpdateReference as
the bench runs them, 0.93 with fixed local maps when `fixed` is given)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from gf_orb_slam_amd import ORBextractor, scene  # noqa: E402
from gf_orb_slam_amd.pipeline import FrontEnd  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
fixed = len(sys.argv) > 4 and sys.argv[4] == "fixed"
stale = float(sys.argv[3]) if len(sys.argv) > 3 else (0.93 if fixed else 0.82)
W = scene.Workload("euroc", B, n_scenes=32, period=32, seed=0, stale_desc=stale)  # as bench.py: distinct frames
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
fe.prof_enable(True)
fe.prof_reset()
for _ in range(steps):
    fe.step()
fe.sync()
rep = fe.prof_report()
tot = sum(v[0] for v in rep.values()) / steps
out = {k: round(v[0] / v[1], 4) for k, v in sorted(rep.items(), key=lambda kv: -kv[1][0])}
print(json.dumps({"batch": B, "ms_per_step_sum": round(tot, 3), "avg_ms": out}))
