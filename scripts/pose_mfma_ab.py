"""PoseOptimization with buildSystem's H / b on MFMA (PO_MFMA build, run with
GF_LIB=gf_orb_slam_amd/diag/libgfslam_pomfma.so) or the product's ordered
VALU sums (default library) against the CPU oracle over many synthetic
problems: how often the LM iteration count, the outlier flags or the inlier
count differ, the largest pose difference, and the bit-identical fraction.
Usage: python scripts/pose_mfma_ab.py [nproblems] [edges]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

import oracle_lib as O  # noqa: E402
from gf_orb_slam_amd.optimizer import Optimizer  # noqa: E402
from gf_orb_slam_amd.synth import synth_pose_problem  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 400
NE = int(sys.argv[2]) if len(sys.argv) > 2 else 80
it_diff = outl_diff = inl_diff = exact = 0
flips = 0
max_rel = 0.0
for seed in range(N):
    _, T0, edges, cam = synth_pose_problem(10000 + seed, NE, noise_px=1.0, outlier_frac=0.1)
    _, _, fx, fy, cx, cy = cam
    Tg, og, ng, ig = Optimizer.pose_opt_edges(T0, edges, fx, fy, cx, cy)
    n = len(edges)
    To, oo, no, io = O.pose_opt(T0, edges["X"], edges["z"], np.arange(n, dtype=np.int32), edges["inv_sigma2"], fx, fy,
                                cx, cy)
    it_diff += int(ig != io)
    inl_diff += int(ng != no)
    d = int((og != oo).sum())
    outl_diff += int(d > 0)
    flips += d
    exact += int(np.array_equal(Tg, To))
    max_rel = max(max_rel, float((np.abs(Tg.astype(np.float64) - To) / np.maximum(1.0, np.abs(To))).max()))
print(json.dumps({"lib": os.environ.get("GF_LIB", "product"), "problems": N, "edges": NE,
                  "iteration_count_differs": it_diff, "inlier_count_differs": inl_diff,
                  "problems_with_outlier_flag_flips": outl_diff, "outlier_flags_flipped": flips,
                  "flags_total": N * NE, "bit_identical_poses": exact, "max_rel_pose_diff": max_rel}))
