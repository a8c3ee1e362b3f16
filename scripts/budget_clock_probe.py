"""Distribution of the front end's budget clock readings (GF_FE_CLOCK) with
budgets far above the step: where each cap's elapsed values fall (ticks of
10 ns). Diagnostic for choosing budgets in tests/test_pipeline_gpu.py."""
import sys

import numpy as np
import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import oracle_lib as O  # noqa: E402
from gf_orb_slam_amd import scene  # noqa: E402
from gf_orb_slam_amd.pipeline import CK, FrontEnd, ck_offsets  # noqa: E402

B, M = int(sys.argv[1]) if len(sys.argv) > 1 else 128, 2000
W = scene.Workload("euroc", B, n_scenes=2, period=32, seed=3, stale_desc=0.93)
frames = W.render_all("cuda").contiguous()
maps = W.build_maps(lambda im: O.extract(im, nfeatures=1000), M)
fe = FrontEnd("euroc", 1000, B, M, 100)
for b in range(B):
    fe.set_map(b, *maps[W.scene_of[b]])
    fe.set_rng(b, 1 + b)
fe.set_source(frames, W.scene_of, W.phase)
T, V = W.boot_state()
fe.bootstrap(T, V, 0.0)
fe.set_budgets(1e9, 1e9)
off = ck_offsets(M, 100)
for k in range(4):
    fe.step()
    c = fe.read("clock")
    nmp = fe.read("nmp")
    st = fe.stats()
    def q(a):
        a = a[a >= 0]
        return [int(x) for x in np.quantile(a, [0, 0.5, 1])] if a.size else None
    viz = np.concatenate([c[b, off["viz"]:off["viz"] + nmp[b]] for b in range(B)])
    am = np.concatenate([c[b, off["am"]:off["am"] + 40] for b in range(B)])
    sel = np.concatenate([c[b, off["sel"]:off["sel"] + (nmp[b] + 63) // 64] for b in range(B)])
    nl = st["nleft"]
    sa = np.concatenate([c[b, off["sa"]:off["sa"] + nl[b]] for b in range(B)])
    bud = np.concatenate([c[b, off["bud"]:off["bud"] + nl[b]] for b in range(B)])
    print(k, {"sofar": q(c[:, CK["sofar"]]), "viz": q(viz), "viz_time": q(c[:, CK["viz_time"]]),
              "mat_online": q(c[:, CK["mat_online"]]), "am_rounds": q(am), "sel": q(sel), "sa": q(sa),
              "sa_sofar": q(c[:, CK["sa_sofar"]]), "bud": q(bud), "branch": np.bincount(st["branch"]).tolist()},
          flush=True)
torch.cuda.synchronize()
