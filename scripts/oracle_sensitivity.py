"""How much do the reference's results depend on the accumulation order of
its small cv::Mat float products? (docs/ORACLE_ASSUMPTIONS.md, A1.)

Runs the CPU oracle chain (tests/oracle_chain.py, the whole tracking step)
free-running over rendered sequences three times — products summed in float
left to right (the parity setting, what the device does), in double with one
rounding (cv::gemm's generic GEMMSingleMul<float,double> path) and as fused
multiply-adds — and compares every step against the float run: last-frame
matches (M3), in-frustum flags (M7) via the matches of the local-map search,
the final map-point assignment and the poses.

Test infrastructure (CPU only). Usage: python scripts/oracle_sensitivity.py [streams] [frames]
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

import oracle_chain as C  # noqa: E402
import oracle_lib as O  # noqa: E402
from gf_orb_slam_amd import scene  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 6
F = int(sys.argv[2]) if len(sys.argv) > 2 else 16
W = scene.Workload("euroc", B, n_scenes=3, period=32, seed=4, tex_size=512)
fr = W.render_all("cpu").numpy()
maps = W.build_maps(lambda im: O.extract(im), 2000)
T, V = W.boot_state()
orc = O.orc()
orc.orc_set_gemm_mode.argtypes = [ctypes.c_int]


def run(mode):
    orc.orc_set_gemm_mode(mode)
    out = []
    for b in range(B):
        ch = C.Chain("euroc", 1000, 2000, 100)
        ch.set_map(*maps[W.scene_of[b]])
        ch.set_rng(1 + b)
        ch.bootstrap(fr[W.scene_of[b], W.phase[b] % W.period], T[b], V[b])
        seq = []
        for k in range(1, F):
            ch.step(fr[W.scene_of[b], (W.phase[b] + k) % W.period])
            st = ch.stats()
            seq.append({"kp2mp": ch.read("kp2mp").copy(), "Tcw": ch.read("Tcw").astype(np.float64),
                        "m3": st["m3"], "inl2": st["inl2"], "branch": st["branch"]})
        out.append(seq)
    orc.orc_set_gemm_mode(0)
    return out


ref = run(0)
res = {"workload": f"{B} rendered euroc sequences x {F - 1} tracked frames (free-running oracle chains)",
       "modes": {}}
for mode, name in ((1, "double accumulation, one rounding"), (2, "fused multiply-add chain")):
    alt = run(mode)
    steps = diff_steps = diff_m3 = 0
    changed = 0
    total = 0
    max_rel = 0.0
    first_div = []
    for b in range(B):
        fd = None
        for k in range(F - 1):
            a, r = alt[b][k], ref[b][k]
            steps += 1
            d = int(np.sum(a["kp2mp"] != r["kp2mp"]))
            changed += d
            total += int(np.sum(r["kp2mp"] >= 0))
            if d:
                diff_steps += 1
                fd = k if fd is None else fd
            diff_m3 += int(a["m3"] != r["m3"])
            max_rel = max(max_rel, float(np.max(np.abs(a["Tcw"] - r["Tcw"]) / np.maximum(1, np.abs(r["Tcw"])))))
        first_div.append(fd)
    res["modes"][name] = {
        "steps_with_any_changed_assignment": f"{diff_steps}/{steps}",
        "changed_assignments": changed, "assignments": total,
        "steps_with_different_M3_count": diff_m3,
        "max_pose_rel_diff": max_rel,
        "first_divergent_step_per_stream": first_div,
    }
print(json.dumps(res, indent=1))
