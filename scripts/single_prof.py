"""One sequence alone (B = 1): per-kernel device time (HIP events per launch)
and the wall time per frame eager and as one HIP graph. Run under
`rocprofv3 --kernel-trace` to see the gaps between the graph's kernels.
Usage: python scripts/single_prof.py [steps] [fixed]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from gf_orb_slam_amd import ORBextractor, scene  # noqa: E402
from gf_orb_slam_amd.pipeline import FrontEnd  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 100
fixed = len(sys.argv) > 2 and sys.argv[2] == "fixed"  # default: the bench's keyframe maps + UpdateReference
W = scene.Workload("euroc", 8, n_scenes=8, period=32, seed=0, stale_desc=0.93 if fixed else 0.82)  # stream 0 as bench.py's single_stream leg
frames = W.render_all("cuda").contiguous()
ex = ORBextractor(1000, 1.2, 8, 1, 20)
M = 2000 if fixed else 2100
if fixed:
    maps = W.build_maps(lambda im: ex(im), M, device="cuda")
else:
    maps = [(g["mp"], g["desc"], g["graph"]) for g in W.build_global_maps(lambda im: ex(im), M, device="cuda")]
fe = FrontEnd("euroc", 1000, 1, M, 100)
fe.set_map(0, *maps[W.scene_of[0]][:2])
if not fixed:
    fe.set_covis(0, maps[W.scene_of[0]][2])
fe.set_rng(0, 1)
fe.set_source(frames, W.scene_of[:1], W.phase[:1])
T, V = W.boot_state()
fe.bootstrap(T[:1], V[:1], 0.0)
for _ in range(3):
    fe.step()
fe.sync()
fe.prof_enable(True)
fe.prof_reset()
for _ in range(steps):
    fe.step()
fe.sync()
rep = fe.prof_report()
fe.prof_enable(False)
tot = sum(v[0] for v in rep.values()) / steps
kern = {k: round(v[0] / v[1] * 1e3, 2) for k, v in sorted(rep.items(), key=lambda kv: -kv[1][0])}
res = {}
for mode in ("eager", "graph"):
    for _ in range(3):
        fe.step()
    if mode == "graph":
        fe.capture_graph()
    fe.sync()
    t1 = time.perf_counter()
    for _ in range(steps):
        fe.step()
    fe.sync()
    res[mode] = round((time.perf_counter() - t1) / steps * 1e3, 4)
print(json.dumps({"ms_per_frame": res, "kernel_us_sum_per_step": round(tot * 1e3, 1), "avg_us": kern}))
