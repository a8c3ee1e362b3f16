"""Latency of the monocular initialiser on the device (gf_initialize_dev):
EuRoC-size two-view scenes (1000-feature frames, ~40% matched), 200 RANSAC
iterations, timed with HIP events on the library's stream. Prints one JSON
line; run under rocprofv3 --kernel-trace --stats for the per-kernel split."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gf_orb_slam_amd.initializer import INIT_RESULT_DTYPE, initialize_batch_device, initialize_device  # noqa: E402
from gf_orb_slam_amd.matcher import default_context  # noqa: E402
from gf_orb_slam_amd.pnp import Rand  # noqa: E402
from gf_orb_slam_amd.synth import synth_two_view  # noqa: E402


def main():
    ctx = default_context()
    dev = torch.device("cuda:0")
    out = {}
    for name, kw in (("general_400of1000", dict(seed=1, n_match=400, n_extra=600)),
                     ("planar_400of1000", dict(seed=1, n_match=400, n_extra=600, planar=True)),
                     ("general_1500of2000", dict(seed=3, n_match=1500, n_extra=500))):
        d = synth_two_view(**kw)
        k1 = torch.from_numpy(d["kps1"].view(np.uint8).reshape(-1, 28).copy()).to(dev)
        k2 = torch.from_numpy(d["kps2"].view(np.uint8).reshape(-1, 28).copy()).to(dev)
        m = torch.from_numpy(d["matches12"].copy()).to(dev)
        rs = torch.from_numpy(Rand(42).state.view(np.uint8).copy()).to(dev)
        s = torch.cuda.current_stream(dev)
        for _ in range(3):
            res, _, _ = initialize_device(ctx, d["K"], k1, k2, m, rs)
        torch.cuda.synchronize()
        reps = 20
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            res, _, _ = initialize_device(ctx, d["K"], k1, k2, m, rs)
        e1.record(s)
        torch.cuda.synchronize()
        r = res.cpu().numpy().view(INIT_RESULT_DTYPE)[0]
        out[name] = {"ms_per_call": e0.elapsed_time(e1) / reps, "ok": int(r["ok"]), "model": int(r["model"]),
                     "nmatches": int(r["nmatches"])}
    # batch: 256 sequences initialising at once (gf_initialize_batch_dev)
    P = 256
    ds = [synth_two_view(seed=100 + i, n_match=400, n_extra=600) for i in range(8)]
    cap1 = max(len(d["kps1"]) for d in ds)
    cap2 = max(len(d["kps2"]) for d in ds)
    k1 = np.zeros((P, cap1, 28), np.uint8)
    k2 = np.zeros((P, cap2, 28), np.uint8)
    mm = np.full((P, cap1), -1, np.int32)
    n1 = np.zeros(P, np.int32)
    n2 = np.zeros(P, np.int32)
    for i in range(P):
        d = ds[i % len(ds)]
        n1[i], n2[i] = len(d["kps1"]), len(d["kps2"])
        k1[i, :n1[i]] = d["kps1"].view(np.uint8).reshape(-1, 28)
        k2[i, :n2[i]] = d["kps2"].view(np.uint8).reshape(-1, 28)
        mm[i, :n1[i]] = d["matches12"]
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    rs = t(np.stack([Rand(7 + i).state.view(np.uint8).reshape(-1) for i in range(P)]))
    args = (ctx, ds[0]["K"], t(k1), t(n1), t(k2), t(n2), t(mm), rs)
    for _ in range(2):
        res, _, _ = initialize_batch_device(*args)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 5
    e0.record(s)
    for _ in range(reps):
        res, _, _ = initialize_batch_device(*args)
    e1.record(s)
    torch.cuda.synchronize()
    r = res.cpu().numpy().view(INIT_RESULT_DTYPE).reshape(P)
    ms = e0.elapsed_time(e1) / reps
    out["batch_256x400of1000"] = {"ms_per_batch": ms, "ms_per_problem": ms / P, "ok": int(r["ok"].sum())}
    print(json.dumps({"initializer": out, "iterations": 200}))


if __name__ == "__main__":
    main()
