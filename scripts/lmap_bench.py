"""Micro-benchmark of the local-mapping matchers on
one GPU: ComputeDistinctiveDescriptors over a whole map, Fuse over a batch of
keyframes, SearchForTriangulation per keyframe pair; kernel time from the
library's HIP-event profiler, the CPU oracle timed on the host beside it.
Prints one JSON object."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import lmap_scenes as S  # noqa: E402
import oracle_lib as O  # noqa: E402
from gf_orb_slam_amd._lib import check, lib, ptr  # noqa: E402
from gf_orb_slam_amd.bow import ORBVocabulary  # noqa: E402
from gf_orb_slam_amd.matcher import FuseProblem, ORBmatcher  # noqa: E402
from gf_orb_slam_amd.orb import default_context  # noqa: E402


def prof(ctx, fn, reps):
    check(lib().gf_prof_enable(ctx.handle, 1))
    check(lib().gf_prof_reset(ctx.handle))
    for _ in range(reps):
        fn()
    check(lib().gf_ctx_sync(ctx.handle))
    out, i = {}, 0
    name, ms, cnt = ctypes.create_string_buffer(64), ctypes.c_double(), ctypes.c_int()
    while lib().gf_prof_report(ctx.handle, i, name, 64, ctypes.byref(ms), ctypes.byref(cnt)) == 0:
        out[name.value.decode()] = (ms.value, cnt.value)
        i += 1
    check(lib().gf_prof_enable(ctx.handle, 0))
    return out


def main():
    ctx = default_context()
    dev = torch.device("cuda:0")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    res = {}
    # ---- ComputeDistinctiveDescriptors over a 200k-point map, 2..30 observations each
    rng = np.random.default_rng(0)
    nmp = 200000
    counts = rng.integers(2, 31, nmp)
    offs = np.zeros(nmp + 1, np.int32)
    offs[1:] = np.cumsum(counts)
    desc = rng.integers(0, 256, (int(offs[-1]), 32), dtype=np.uint8)
    dd, do = t(desc), t(offs)
    db = torch.zeros(nmp, dtype=torch.int32, device=dev)
    dout = torch.zeros((nmp, 32), dtype=torch.uint8, device=dev)
    run = lambda: check(lib().gf_distinctive_descriptors_dev(ctx.handle, nmp, ptr(dd), ptr(do), ptr(db), ptr(dout),
                                                             int(offs[-1]), ctx.stream))
    run()
    pr = prof(ctx, run, 10)
    us = sum(1e3 * v[0] / v[1] for k, v in pr.items() if k.startswith("k_distinctive"))
    ns = 20000
    t0 = time.perf_counter()
    O.distinctive_descriptors(desc[:offs[ns]], offs[:ns + 1])
    cpu = time.perf_counter() - t0
    pairs = int((counts.astype(np.int64) ** 2).sum())
    res["distinctive"] = {"points": nmp, "observations": int(offs[-1]), "kernel_us": round(us, 1),
                          "points_per_s": round(nmp / (us * 1e-6)), "hamming_pairs_per_s": round(pairs / (us * 1e-6)),
                          "hbm_bytes": int(32 * offs[-1] + 4 * (nmp + 1) + 36 * nmp),
                          "cpu_points_per_s_1core": round(ns / cpu)}
    # ---- Fuse: 64 keyframes x 3000 candidates
    scs = [S.fuse_scene(100 + i, nmp=2500, nkp=1000, dup=500) for i in range(8)]
    probs, keep = [], []
    for i in range(64):
        sc = scs[i % 8]
        kf = sc["kf"]
        bufs = [t(kf.mvKeysUn.view(np.uint8)), t(kf.mDescriptors), t(sc["kf_mp"]), t(sc["kf_bad"]),
                t(sc["mps"].view(np.uint8)), t(sc["mp_desc"]), t(sc["skip"]), t(sc["ids"]),
                torch.zeros(len(sc["mps"]) * 3, dtype=torch.int32, device=dev),
                torch.zeros(1, dtype=torch.int32, device=dev)]
        keep += bufs
        probs.append(FuseProblem.make(sc["Tcw"], sc["Ow"], bufs, kf.N, len(sc["mps"]), 3.0))
    arr = (FuseProblem * len(probs))(*probs)
    info = scs[0]["info"]
    run = lambda: check(lib().gf_fuse_dev(ctx.handle, ctypes.byref(info), len(probs), arr, ctx.stream))
    run()
    p = prof(ctx, run, 10)["k_fuse"]
    us = 1e3 * p[0] / p[1]
    sc = scs[0]
    kf = sc["kf"]
    t0 = time.perf_counter()
    for _ in range(5):
        O.fuse(sc["info"], sc["Tcw"], sc["Ow"], kf.mvKeysUn, kf.mDescriptors, sc["kf_mp"], sc["kf_bad"], sc["mps"],
               sc["mp_desc"], sc["skip"], sc["ids"], 3.0)
    cpu = (time.perf_counter() - t0) / 5
    res["fuse"] = {"keyframes": len(probs), "candidates_per_kf": len(sc["mps"]), "keypoints_per_kf": kf.N,
                   "kernel_us": round(us, 1), "us_per_keyframe": round(us / len(probs), 2),
                   "cpu_us_per_keyframe_1core": round(cpu * 1e6, 1)}
    # ---- SearchForTriangulation: one keyframe pair per launch (host entry)
    gfv = lambda voc, d, levelsup=2: ORBVocabulary(voc).transform(d, levelsup)[2]
    a, b, F, s2 = S.triangulation_pair(3, 1000, 1000, fv=gfv)
    m = ORBmatcher(0.6, True)
    run = lambda: m.SearchForTriangulation(a, b, F, s2)
    run()
    p = prof(ctx, run, 20)["k_search_tri"]
    us = 1e3 * p[0] / p[1]
    tup = lambda s: ((s[0].nodes, s[0].start, s[0].feats),) + s[1:]
    t0 = time.perf_counter()
    for _ in range(20):
        O.search_triangulation(True, tup(a), tup(b), F, s2)
    cpu = (time.perf_counter() - t0) / 20
    res["triangulation"] = {"keypoints": [1000, 1000], "kernel_us": round(us, 1),
                            "cpu_us_1core": round(cpu * 1e6, 1), "note": "one workgroup per pair; batch pairs to fill the chip"}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
