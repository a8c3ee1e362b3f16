"""Per-kernel device time of one front-end group alone (no overlapping
groups): B sequences of the bench workload, HIP events per launch.
Usage: python scripts/kernel_times.py [B] [steps] [stale]  (stale map-descriptor
fraction, default 0.93: the bench's config-2 regime)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from gf_orb_slam_amd import ORBextractor, scene  # noqa: E402
from gf_orb_slam_amd.pipeline import FrontEnd  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
stale = float(sys.argv[3]) if len(sys.argv) > 3 else 0.93
W = scene.Workload("euroc", B, n_scenes=8, period=32, seed=0, stale_desc=stale)
frames = W.render_all("cuda").contiguous()
ex = ORBextractor(1000, 1.2, 8, 1, 20)
maps = W.build_maps(lambda im: ex(im), 2000, device="cuda")
fe = FrontEnd("euroc", 1000, B, 2000, 100)
for b in range(B):
    fe.set_map(b, *maps[W.scene_of[b]])
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
