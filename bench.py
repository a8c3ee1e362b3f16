#!/usr/bin/env python3
"""GF-ORB-SLAM front-end benchmark (BASELINE.json metric).

Metric: front-end fps (extract + match + GF-select) @ 752x480 / 1000 feats,
plus pose-opt ms/iter. Config 2 (EuRoC camera, 1000 feats, GF budget 100,
2000-point local maps) on rendered sequences: one step = one frame of each
of B independent tracked sequences through libgfslam's batched front end
(gf_frontend_step: Tracking::GrabImage in the WORKING state — extraction,
TrackWithMotionModel, TrackLocalMap with the GF branch, motion model,
next-frame prediction, SearchAdditionalMatchesInFrame, hand-over to the last
frame). Every stream carries its pose, velocity, matches, map stamps and
std::rand() state from frame to frame. value = frames of all ranks / wall
time, frames resident in HBM.

Multi-GPU (config 5): one process per GPU. `--gpus N` launches N ranks itself
(torch.distributed.run) when it is not already running under a launcher.
Rank 0 builds the world (scenes, vocabulary, local maps) and broadcasts it
over RCCL (gf_dist_*, xGMI); each rank then tracks its own sequences (its own
phases of the loops), weak scaling, no per-frame communication.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Algorithmic bytes per frame for the extraction kernels,
# from the level sizes: P = sum of pyramid pixels.
LEVELS = {"euroc": [(752, 480), (627, 400), (522, 333), (435, 278), (363, 231), (302, 193), (252, 161), (210, 134)],
          "tum": [(640, 480), (533, 400), (444, 333), (370, 278), (309, 231), (257, 193), (214, 161), (179, 134)]}


def kernel_bytes(camera: str, nfeat: int) -> dict:
    px = [w * h for w, h in LEVELS[camera]]
    P, P0, P7 = sum(px), px[0], px[-1]
    return {
        "k_pyramid": P,                   # read level 0, write levels 1.. (the levels between stay in LDS)
        "k_blur_fast": 3 * P,             # read every level, write blurred level + FAST score map
        "k_describe": 60 * nfeat,         # 32 B descriptor + 28 B keypoint out
        "k_describe_planes": 2 * P + 60 * nfeat,  # + both planes read once (IC_Angle level, rBRIEF blurred level)
        "extract_total": P + 3 * P + 2 * P + 60 * nfeat,
    }


class _StdoutToStderr:
    """Send fd 1 to fd 2 for a block: RCCL prints its version banner on
    stdout at communicator init, and the bench's stdout is one JSON line."""

    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)
        return self

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)
        return False


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


# ------------------------------------------------------------- CPU baseline
def _chain_worker(args) -> tuple:
    """One host core tracking one sequence on the CPU oracle chain
    (oracle/chain.cpp, timing build); no GPU."""
    camera, nfeat, nmap, budget, fps, m, frames, T, V, seed, budget_s, lib = args
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ["GF_ORACLE_LIB"] = lib
    import oracle_chain as C

    ch = C.Chain(camera, nfeat, nmap, budget, fps=fps)
    ch.set_map(m[0], m[1])
    if len(m) > 2:
        ch.set_covis(m[2])
    ch.set_rng(seed)
    ch.bootstrap(frames[0], T, V)
    times, stages = [], []
    t0 = time.perf_counter()
    k = 0
    while time.perf_counter() - t0 < budget_s:
        k += 1
        t1 = time.perf_counter()
        ch.step(frames[k % len(frames)])
        times.append(time.perf_counter() - t1)
        stages.append(ch.timings())
    return k, time.perf_counter() - t0, times, np.array(stages)


def _physical_cpus(cpus: list) -> list:
    """One logical CPU per physical core among `cpus` (sysfs topology; the
    first sibling of each core), in CPU order."""
    seen, out = set(), []
    for c in sorted(cpus):
        try:
            base = f"/sys/devices/system/cpu/cpu{c}/topology/"
            key = (open(base + "physical_package_id").read().strip(), open(base + "core_id").read().strip())
        except OSError:
            key = ("?", str(c))
        if key not in seen:
            seen.add(key)
            out.append(c)
    return out


def _host_physical_cores() -> int:
    try:
        return len(_physical_cpus(list(range(os.cpu_count() or 1))))
    except Exception:
        return os.cpu_count() or 1


def cpu_share() -> list:
    """The CPUs this job may use, one per physical core: the affinity set,
    capped at the job's CPU share when the environment states one
    (GF_CPU_SHARE, else OMP_NUM_THREADS: a one-GPU job on the GPU box is
    granted 16 CPUs, which is also the node's 128 physical cores / 8 GPUs)."""
    aff = sorted(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else list(range(os.cpu_count() or 1))
    phys = _physical_cpus(aff)
    cap = os.environ.get("GF_CPU_SHARE") or os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit() and int(cap) > 0:
        phys = phys[:int(cap)]
    return phys or aff[:1]


def _pinned_chain_worker(args) -> tuple:
    cpu, job = args
    try:
        os.sched_setaffinity(0, {cpu})
    except (AttributeError, OSError):
        pass
    return _chain_worker(job)


def cpu_baseline(camera, nfeat, nmap, budget, fps, maps, W, frames_host, budget_s=12.0) -> dict:
    """The oracle chain (CPU restatement of the same step) on a bounded sample
    of the same workload: (i) one core, one sequence — the baseline value —
    with median / p90 per frame and per stage; (ii) every core of the job's
    CPU share (cpu_share: one worker process per physical core, each pinned
    to its core with sched_setaffinity), one independent sequence per process
    (throughput). Timing build of the oracle: -O3 -march=x86-64-v3 with
    vectorisation (oracle/liboracle_fast.so; the parity build is
    -fno-tree-vectorize)."""
    import multiprocessing as mp_
    import platform

    lib = os.path.join(ROOT, "oracle", "liboracle_fast.so")
    if not os.path.exists(lib):
        lib = os.path.join(ROOT, "oracle", "liboracle.so")

    def job(b, secs):
        s = W.scene_of[b]
        seq = np.stack([frames_host[s][(W.phase[b] + k) % W.period] for k in range(W.period)])
        T, V = W.boot_state()
        return (camera, nfeat, nmap, budget, fps, maps[s], seq, T[b], V[b], 1 + b, secs, lib)

    cpus = cpu_share()
    n, dt, times, stages = _pinned_chain_worker((cpus[0], job(0, budget_s)))
    t = np.sort(np.asarray(times)) * 1e3
    names = ["extract", "track_motion_model", "frame_info", "local_map_search", "pose_opt_2",
             "predict_next", "additional_matches"]
    st = np.asarray(stages) * 1e3
    out = {"value": round(n / dt, 3), "unit": "frames/s", "cores": 1, "kind": "port",
           "sample": f"{n} consecutive frames of one rendered {camera} sequence ({nfeat} feats, "
                     f"{'keyframe map of %d points, UpdateReference every frame' % nmap if len(maps[0]) > 2 else '%d-point local map' % nmap}, "
                     f"GF budget {budget}), full tracking step per frame on the C++ oracle chain, "
                     f"1 thread, {dt:.1f} s",
           "build": os.path.basename(lib),
           "ms_per_frame_median": round(float(np.median(t)), 2),
           "reference_published": "the reference's own figure is ~11-16 ms average per-frame tracking latency on "
                                  "EuRoC (BASELINE.md §1, read off a plot, hardware not stated); this port's "
                                  "extraction is a scalar restatement of OpenCV's (no SIMD FAST/blur/resize), so the "
                                  "single-core figure is a port of the algorithm, not the reference binary",
           "ms_per_frame_p90": round(float(t[int(0.9 * (len(t) - 1))]), 2),
           "stages_ms_median": {k: round(float(np.median(st[:, i])), 3) for i, k in enumerate(names)}}
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            cpu_model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), "")
    except OSError:
        pass
    w = len(cpus)
    ctx = mp_.get_context("spawn")  # fresh interpreters: the workers never touch the GPU
    with ctx.Pool(w) as pool:
        res = pool.map(_pinned_chain_worker, [(cpus[i], job(1 + i, budget_s * 0.6)) for i in range(w)])
    frames = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    phys = _host_physical_cores()
    out["all_cores"] = {"value": round(frames / wall, 2), "unit": "frames/s", "cores": w,
                        "pinned_cpus": cpus,
                        "sample": f"{frames} frames, one sequence per process, one process pinned per physical "
                                  f"core, {wall:.1f} s",
                        "share_note": "every core of this job's CPU share (the GPU box grants a one-GPU job 16 "
                                      "CPUs; the node has %d physical cores for its GPUs)" % phys}
    out["host"] = {"nproc": os.cpu_count(), "physical_cores": phys, "cpu_model": cpu_model or platform.processor()}
    return out


# ------------------------------------------------------------- local BA leg
def schur_flops(prob: dict) -> float:
    """Algorithmic flops of one Schur contraction (k_ba_gemm) for one LBA
    window: per map point with k edges to local (free) keyframes, the k(k+1)/2
    6x6 blocks W_i Hpl_j^T (3 products each) and the k 6-vectors Hpl_i db."""
    free = prob["kf_kind"][prob["edge_kf"]] == 0
    k = np.bincount(prob["edge_pt"][free], minlength=len(prob["pt_pos"])).astype(np.float64)
    return float((k * (k + 1) / 2 * 36 * 3 * 2 + k * 6 * 3 * 2).sum())


def schur_mfma_count(prob: dict) -> int:
    """v_mfma_f64_16x16x4f64 issued by one Schur contraction of one window:
    the (k-step, 16x16 tile) pairs whose column-tile masks are both set, the
    rule the library builds its task list / masks with (csrc/ba.hip,
    gf_ba_plan_create). Executed flops = count x 2048."""
    kind = np.asarray(prob["kf_kind"])
    col = np.full(len(kind), -1)
    col[kind == 0] = np.arange(int((kind == 0).sum()))
    n = 6 * int((kind == 0).sum())
    npad = ((n + 1 + 15) // 16) * 16
    nt, tdb = npad // 16, n >> 4
    npts = len(prob["pt_pos"])
    steps = max(1, (3 * npts + 3) // 4)
    mask = np.zeros(steps, np.int64)
    ept, ekf = np.asarray(prob["edge_pt"]), np.asarray(prob["edge_kf"])
    c = col[ekf]
    sel = c >= 0
    bits = (1 << ((6 * c[sel]) >> 4)) | (1 << ((6 * c[sel] + 5) >> 4))
    for r in range(3):
        np.bitwise_or.at(mask, (3 * ept[sel] + r) // 4, bits)
    tiles = [(a, b) for a in range(nt) for b in range(a + 1)] + [(a, tdb) for a in range(tdb)]
    mb = mask | (1 << tdb)
    cnt = 0
    for ti, tj in tiles:
        cnt += int(((mask != 0) & ((mask >> ti) & 1 == 1) & ((mb >> tj) & 1 == 1)).sum())
    return cnt


def lba_leg(batch: int, repeats: int = 3, cpu: bool = True) -> dict:
    """Config 4: LocalBundleAdjustment on synthetic 20-keyframe x
    3000-point windows, `batch` independent windows solved together on the
    device (inputs resident), plus the single-window latency."""
    import torch

    from gf_orb_slam_amd._lib import check, lib
    from gf_orb_slam_amd.optimizer import LocalBAPlan
    from gf_orb_slam_amd.synth import synth_lba_problem

    out = {"workload": "config 4: LocalBundleAdjustment, 20 keyframes (17-19 local) x 3000 map points, ~15k edges",
           "dtype": "f64"}
    for B in sorted({1, batch}):
        probs = [synth_lba_problem(1000 + i, 20, 3000) for i in range(B)]
        plan = LocalBAPlan(probs)
        plan.solve()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(repeats):
            steps = plan.solve()
        dt = (time.perf_counter() - t0) / repeats
        res = plan.results()
        iters = np.array([r[3] for r in res], np.float64)
        check(lib().gf_prof_enable(plan.ctx.handle, 1))
        check(lib().gf_prof_reset(plan.ctx.handle))
        plan.solve()
        prof = {}
        i = 0
        name = ctypes.create_string_buffer(64)
        while True:
            ms, cnt = ctypes.c_double(), ctypes.c_int()
            if lib().gf_prof_report(plan.ctx.handle, i, name, 64, ctypes.byref(ms), ctypes.byref(cnt)) != 0:
                break
            prof[name.value.decode()] = (ms.value, cnt.value)
            i += 1
        check(lib().gf_prof_enable(plan.ctx.handle, 0))
        plan.close()
        g_ms, g_n = prof.get("k_ba_gemm", (0.0, 1))
        flops = sum(schur_flops(p) for p in probs)
        entry = {"problems": B, "ms_per_batch": round(dt * 1e3, 3), "solves_per_s": round(B / dt, 2),
                 "ms_per_solve_amortized": round(dt * 1e3 / B, 4), "steps": steps,
                 "lm_iterations": [round(float(x), 2) for x in iters.mean(0)],
                 "ms_per_lm_iteration": round(dt * 1e3 / float(iters.sum(1).mean()), 4),
                 "kernels": {k: {"avg_us": round(v[0] / max(v[1], 1) * 1e3, 2), "launches": v[1]}
                             for k, v in prof.items()}}
        if g_ms > 0:
            tf = flops / (g_ms / g_n / 1e3) / 1e12
            xflops = 2048.0 * sum(schur_mfma_count(p) for p in probs)
            xtf = xflops / (g_ms / g_n / 1e3) / 1e12
            entry["schur_gemm"] = {"bound": "mfma", "achieved": round(tf, 4), "peak": 78.6, "unit": "TFLOP/s",
                                   "frac": round(tf / 78.6, 6), "algorithmic_flops_per_launch": flops,
                                   "executed_flops_per_launch": xflops, "executed_tflops": round(xtf, 3),
                                   "executed_frac": round(xtf / 78.6, 5),
                                   "kernel": "k_ba_spgemm (task list)" if B <= 8 else "k_ba_gemm (dense split-K)",
                                   "note": "f64 MFMA 16x16x4; peak = AMD spec FP64 matrix (not measured here); "
                                           "executed = whole 16x16x4 tiles the masks select"}
            try:
                pm = json.load(open(os.path.join(ROOT, "profiles", "r04", "pmc_lba_mfma.json")))
                if pm.get("batch") == B:
                    entry["schur_gemm"]["mfma_busy_pmc"] = round(pm["mfma_busy_fraction"], 5)
                    entry["schur_gemm"]["mfma_busy_source"] = "profiles/r04/pmc_lba_mfma.json"
            except (OSError, ValueError, KeyError):
                pass
        out["batch_%d" % B] = entry
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib

        p = synth_lba_problem(1000, 20, 3000)
        n, t0 = 0, time.perf_counter()
        while time.perf_counter() - t0 < 5.0:
            oracle_lib.local_ba(p)
            n += 1
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(n / dt, 3), "unit": "solves/s", "cores": 1, "kind": "port",
                               "sample": f"{n} solves of one config-4 window, 1 thread, {dt:.1f} s (dense LL^T in "
                                         f"place of CHOLMOD)"}
    return out


# ------------------------------------------------------------- config 3 leg
def config3_leg(local: int, batch: int, groups: int, steps: int, warmup: int) -> dict:
    """BASELINE config 3 (TUM RGB-D 640x480, 2000 features, GF budget 160 +
    PoseOptimization) on this GPU: `batch` rendered sequences in `groups`
    gated front ends, 3000-point keyframe-built local maps with 93% stale
    descriptors (the GF regime: runActiveMapMatching on most frames), timed
    like the headline; the dominant §8d-priced kernel's roofline."""
    import torch

    from gf_orb_slam_amd import ORBextractor, scene
    from gf_orb_slam_amd.orb import Context
    from gf_orb_slam_amd.pipeline import STATS, FrontEnd, chain_extraction

    cam, nfeat, budget, nmap, stale = "tum", 2000, 160, 3000, 0.93
    B, G = batch, max(1, groups)
    Bg = B // G
    W = scene.Workload(cam, B, n_scenes=8, period=32, seed=1, stale_desc=stale)
    ex = ORBextractor(nfeat, 1.2, 8, 1, 20)
    maps = W.build_maps(lambda im: ex(im), nmap, device=f"cuda:{local}")
    frames = W.render_all(f"cuda:{local}").contiguous()
    T, V = W.boot_state()
    fes = []
    for g in range(G):
        sl = slice(g * Bg, (g + 1) * Bg)
        fe = FrontEnd(cam, nfeat, Bg, nmap, budget, ctx=Context(local))
        for b in range(Bg):
            fe.set_map(b, *maps[W.scene_of[g * Bg + b]])
            fe.set_rng(b, 7 + g * Bg + b)
        fe.set_source(frames, W.scene_of[sl], W.phase[sl])
        fe.bootstrap(T[sl], V[sl], 0.0)
        fes.append(fe)
    gates = chain_extraction(fes)
    for _ in range(warmup):
        for fe in fes:
            fe.step()
    for fe in fes:
        fe.sync()
        fe.write("hist", np.zeros((fe.B, 8), np.int32))
        fe.prof_enable(True)
        fe.prof_reset()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        for fe in fes:
            fe.step()
    for fe in fes:
        fe.sync()
    dt = time.perf_counter() - t0
    prof = {}
    for fe in fes:
        for k, (ms, cnt) in fe.prof_report().items():
            a = prof.setdefault(k, [0.0, 0])
            a[0] += ms
            a[1] += cnt
        fe.prof_enable(False)
    th = np.concatenate([fe.read("hist") for fe in fes]).astype(np.int64)
    st = [fe.stats() for fe in fes]
    final = {k: np.concatenate([x[k] for x in st]) for k in STATS}
    for fe in fes:
        fe.close()
    del gates
    kb = kernel_bytes(cam, nfeat)
    ldets = float(th[:, 6].sum())
    work = {"k_pyramid": kb["k_pyramid"] * Bg, "k_blur_fast": kb["k_blur_fast"] * Bg,
            "k_describe": kb["k_describe"] * Bg}
    if "k_active_match" in prof:
        work["k_active_match"] = 224.0 * ldets / max(prof["k_active_match"][1], 1)
    priced = {}
    for k, units in work.items():
        if k not in prof:
            continue
        ms = prof[k][0] / prof[k][1]
        if k == "k_active_match" and "k_active_match_overflow" in prof:
            ms = (prof[k][0] + prof["k_active_match_overflow"][0]) / prof[k][1]
        ach = units / (ms / 1e3) / 1e9
        priced[k] = {"kernel": k, "bound": "hbm", "achieved": round(ach, 3), "peak": 8000.0, "unit": "GB/s",
                     "frac": round(ach / 8000.0, 6), "algorithmic_bytes_per_launch": units,
                     "avg_launch_ms": round(ms, 4), "launches": prof[k][1]}
    dom = max(priced, key=lambda k: prof[k][0])
    ext_ms = sum(prof[k][0] for k in ("k_pyramid", "k_blur_fast", "k_fast_cells", "k_select", "k_describe")
                 if k in prof)
    return {"workload": f"config 3: tum 640x480, {nfeat} feats, GF budget {budget}, {nmap}-point keyframe-built "
                        f"local maps ({stale:.2f} stale descriptors), {B} sequences in {G} gated groups, "
                        f"PoseOptimization twice per frame",
            "frames_per_s": round(B * steps / dt, 1), "ms_per_step": round(dt / steps * 1e3, 3), "steps": steps,
            "warmup": warmup, "roofline": {**priced[dom], "others": {k: v for k, v in priced.items() if k != dom}},
            "extraction_algorithmic_GBps": round(kb["extract_total"] * B * steps / (ext_ms / 1e3) / 1e9, 1)
            if ext_ms else None,
            "branch_mix_timed": {"leftovers_only": int(th[:, 1].sum()), "search_by_projection": int(th[:, 2].sum()),
                                 "active_matching": int(th[:, 3].sum()), "nothing_to_match": int(th[:, 4].sum())},
            "logdets_per_frame": round(ldets / (B * steps), 1),
            "mean_inliers": round(float(final["inl2"].mean()), 1),
            "lost_frames_last_step": int((final["flags"] & 4 != 0).sum()),
            "kernels": {k: {"avg_ms": round(v[0] / max(v[1], 1), 4), "launches": v[1]} for k, v in prof.items()}}


# ------------------------------------------------------------- output line
LINE_CAP = 8000


def compact_line(out: dict, detail: str) -> str:
    """The one JSON line the driver parses: the contract fields, the dominant
    kernel's roofline plus up to four other priced kernels as flat entries, the
    CPU baseline, a few scalar legs. Everything else is in `detail`."""
    roof = out.get("roofline", {})
    keep = ("kernel", "bound", "achieved", "peak", "unit", "frac", "traffic", "timing", "avg_launch_ms",
            "avg_launch_ms_events", "algorithmic_bytes_per_launch", "algorithmic_flops_per_launch", "launches")
    r = {k: roof[k] for k in keep if k in roof}
    r["frames_per_launch"] = roof.get("frames_per_launch")
    others = roof.get("other_kernels", {})
    order = sorted(others, key=lambda k: -others[k].get("avg_launch_ms", 0))[:4]
    r["others"] = {k: {f: others[k].get(f) for f in ("bound", "achieved", "unit", "frac", "avg_launch_ms",
                                                       "traffic")} for k in order}
    cb = out.get("cpu_baseline")
    line = {k: out[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                "higher_is_better", "scaling", "vs_baseline", "dtype")}
    line["data"] = "synthetic: rendered EuRoC-like sequences, keyframe maps; no dataset"
    c = out["config"]
    line["config"] = {"workload": "config 2: euroc 752x480, 1000 feats, GF budget 100, full GrabImage step "
                                  "(extract, match, GF select, 2x PoseOptimization) with UpdateReference",
                      "sequences_per_gpu": c.get("sequences_per_gpu"), "stream_groups": c.get("stream_groups"),
                      "distinct_frames_per_step": c.get("distinct_frames_per_step"),
                      "parallelism": c.get("parallelism")}
    if out.get("n_gpus", 1) > 1 or out.get("ranks", {}).get("transport") == "host":
        line["ranks"] = {k: out["ranks"][k] for k in ("world", "communicator_world", "transport", "devices_used",
                                                      "frames_per_s", "min_frames_per_s", "max_frames_per_s",
                                                      "max_over_min_ms")}
        line["startup_checksums_equal"] = out.get("startup", {}).get("checksums_equal_across_ranks")
    line["roofline"] = r
    if cb:
        line["cpu_baseline"] = {k: cb.get(k) for k in ("value", "unit", "cores", "kind", "vs_published")}
        line["cpu_baseline"]["sample"] = cb.get("sample", "")[:200]
        if "all_cores" in cb:
            line["cpu_baseline"]["all_cores"] = {k: cb["all_cores"].get(k) for k in ("value", "cores")}
    extra = {}
    if "single_stream" in out:
        extra["single_stream_ms_per_frame"] = out["single_stream"].get("ms_per_frame")
    if "pose_opt" in out:
        extra["pose_opt_ms_per_iter"] = out["pose_opt"].get("ms_per_iter")
    lba = out.get("local_ba", {})
    if "batch_1" in lba:
        extra["local_ba_ms_per_window"] = lba["batch_1"].get("ms_per_batch")
    if "config3" in out:
        extra["config3_frames_per_s"] = out["config3"].get("frames_per_s")
    if "budgets_on" in out:
        extra["budgets_on_frames_per_s"] = out["budgets_on"].get("frames_per_s")
    line["legs"] = extra
    line["detail"] = detail
    s = json.dumps(line)
    if len(s) > LINE_CAP:  # never exceed the cap: drop the optional parts first
        for drop in ("legs", "others"):
            if drop == "others":
                line["roofline"].pop("others", None)
            else:
                line.pop(drop, None)
            s = json.dumps(line)
            if len(s) <= LINE_CAP:
                break
    return s


# ------------------------------------------------------------- kernel table
def _under_profiler() -> bool:
    """True inside a rocprofv3 (or older rocprof) run: no nested profiler."""
    return (any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ)
            or "rocprof" in os.environ.get("LD_PRELOAD", ""))


def _kname(raw: str) -> str:
    return raw.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0].split("<")[0]


def rocprof_kernel_table(args) -> tuple:
    """Per-kernel dispatch durations of the headline timed region from a
    rocprofv3 kernel trace of this script run as a child process (the same
    workload and step counts, the other legs off, no HIP events in the timed
    region): HIP events on a stream that shares a hardware queue with the
    other groups' streams count the wait behind their kernels, the dispatch
    timestamps do not. The timed region is the dispatches from the first
    k_fe_begin of the timed steps to the last k_fe_end of them (one per group
    and step). -> ({kernel: [durations ns]}, queues used, note)."""
    import glob
    import shutil
    import tempfile

    exe = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(exe):
        return None, None, "rocprofv3 not found"
    d = tempfile.mkdtemp(prefix="gf_bench_kt_", dir="/tmp")
    child = sys.argv[1:] + ["--kernels-child", "--no-prof-timed", "--no-cpu-baseline", "--single-stream-steps", "0",
                            "--lba-batch", "0", "--config3-steps", "0", "--pcie-steps", "0", "--budget-steps", "0",
                            "--isolated-steps", "0", "--kernel-times", "events"]
    cmd = [exe, "--kernel-trace", "--stats", "--output-format", "csv", "-d", d, "-o", "run", "--", sys.executable,
           os.path.abspath(__file__)] + child
    try:
        r = subprocess.run(cmd, cwd=d, env=dict(os.environ, TMPDIR="/tmp"), stdout=subprocess.DEVNULL,
                           stderr=subprocess.PIPE, timeout=600)
    except subprocess.TimeoutExpired:
        return None, None, "rocprofv3 child timed out"
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if r.returncode != 0 or not tr:
        return None, None, "rocprofv3 child failed (exit %d): %s" % (r.returncode, r.stderr.decode()[-300:])
    import csv

    rows = list(csv.DictReader(open(tr[0])))
    keep = getattr(args, "kernel_trace_dir", None)
    if keep:  # the child's rocprof files (its --stats summary and trace) beside the bench output
        os.makedirs(keep, exist_ok=True)
        for f_ in glob.glob(os.path.join(d, "**", "*.csv"), recursive=True):
            shutil.copy(f_, os.path.join(keep, os.path.basename(f_)))
    shutil.rmtree(d, ignore_errors=True)
    G, W, K = max(1, args.groups), args.warmup, args.steps
    beg = sorted(int(x["Start_Timestamp"]) for x in rows if _kname(x["Kernel_Name"]) == "k_fe_begin")
    end = sorted(int(x["End_Timestamp"]) for x in rows if _kname(x["Kernel_Name"]) == "k_fe_end")
    if len(beg) < (W + K) * G or len(end) < (W + K) * G:
        return None, None, "timed region not found in the trace"
    t0, t1 = beg[W * G], end[(W + K) * G - 1]
    acc, queues = {}, set()
    for x in rows:
        a, b = int(x["Start_Timestamp"]), int(x["End_Timestamp"])
        if a >= t0 and b <= t1:
            acc.setdefault(_kname(x["Kernel_Name"]), []).append(b - a)
            queues.add(x.get("Queue_Id"))
    if keep:  # the timed region's table (the figures `kernels` reports), as scripts/trace_timed.py writes it
        tot = sum(sum(v) for v in acc.values())
        with open(os.path.join(keep, "kernel_stats_timed.csv"), "w", newline="") as fh:
            w = csv.writer(fh)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
                w.writerow([k, len(v), sum(v), round(sum(v) / len(v), 1), round(100.0 * sum(v) / tot, 2), min(v),
                            max(v)])
    return acc, len(queues), None


# ------------------------------------------------------------- main
def build_world(cam: str, B: int, S: int, period: int, nfeat: int, nmap: int, device: int, stale: float,
                refmap: bool, n_kf: int):
    """Rank 0: the scenes of the loops and each scene's map (keyframes
    extracted with the product extractor on this GPU): with refmap a keyframe
    map (points, descriptors, covisibility graph) whose local map
    Tracking::UpdateReference assembles every frame, else one fixed
    keyframe-built local map."""
    from gf_orb_slam_amd import ORBextractor, scene

    W0 = scene.Workload(cam, B, n_scenes=S, period=period, seed=0, stale_desc=stale)
    ex = ORBextractor(nfeat, 1.2, 8, 1, 20)
    if refmap:
        gm = W0.build_global_maps(lambda im: ex(im), nmap, n_kf=n_kf, device=f"cuda:{device}")
        return W0.scenes, [(g["mp"], g["desc"], g["graph"], g["kf_kps"], g["kf_desc"]) for g in gm]
    return W0.scenes, W0.build_maps(lambda im: ex(im), nmap, device=f"cuda:{device}")


def load_map(fe, b: int, m, with_points: bool = True):
    """Stream b's map: points + descriptors (skipped when another rank's
    broadcast supplies them), then its keyframe graph if the world has one."""
    if with_points:
        fe.set_map(b, m[0], m[1])
    if len(m) > 2:
        fe.set_covis(b, m[2])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=1024, help="independent sequences per GPU")
    ap.add_argument("--groups", type=int, default=4,
                    help="stream groups per GPU, each a front end on its own HIP stream (their kernels overlap; 4 x 256 measured best in r03: 95.9k vs 89.5k frames/s for 2 x 512)")
    ap.add_argument("--no-gate", action="store_true",
                    help="let the groups' extraction stages overlap (default: chained, one at a time)")
    ap.add_argument("--gate-stage", type=int, default=None,
                    help="extraction stage after which the gate releases the next group (0 resize .. 4 describe; "
                         "default: the library's, after describe)")
    ap.add_argument("--track-priority", action="store_true",
                    help="each group's tracking kernels on a high-priority stream of their own "
                         "(gf_frontend_set_track_priority; measured slower on MI355X: 70k vs 89k frames/s)")
    ap.add_argument("--camera", default="euroc")
    ap.add_argument("--nfeatures", type=int, default=1000)
    ap.add_argument("--gf-budget", type=int, default=100)
    ap.add_argument("--map", type=int, default=None,
                    help="map points per sequence: the keyframe map (default 2100, local maps of ~2000 points "
                         "assembled from it) or, with --fixed-map, the fixed local map (default 2000)")
    ap.add_argument("--fixed-map", action="store_true",
                    help="one fixed local map per sequence instead of UpdateReference over a keyframe map")
    ap.add_argument("--keyframes", type=int, default=24, help="keyframes of each scene's map (UpdateReference mode)")
    ap.add_argument("--stale-desc", type=float, default=None,
                    help="fraction of map points with a stale (random) descriptor; the defaults (0.82 keyframe map, "
                         "0.93 fixed map) give config 2's regime of SURVEY §8d: ~60 motion-model matches vs GF "
                         "budget 100, runActiveMapMatching every frame (scene.build_map / build_global_map)")
    ap.add_argument("--scenes", type=int, default=32,
                    help="rendered rooms (each its own keyframe map); 32 rooms x 32-frame loops give the 1024 "
                         "sequences of a step 1024 distinct frames")
    ap.add_argument("--period", type=int, default=32, help="frames per loop of the rendered trajectory")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--lba-batch", type=int, default=64, help="local-BA windows solved together (0: skip)")
    ap.add_argument("--single-stream-steps", type=int, default=40,
                    help="also time one sequence alone (per-frame latency, HIP graph replay)")
    ap.add_argument("--isolated-steps", type=int, default=5,
                    help="also time the priced kernel with one group running alone")
    ap.add_argument("--budget-steps", type=int, default=5,
                    help="also time the step with the reference's time budgets on (gf_set_budgets)")
    ap.add_argument("--pcie-steps", type=int, default=5,
                    help="also time one group with the frames handed over from host memory")
    ap.add_argument("--hw-queues", type=int, default=0,
                    help="GPU_MAX_HW_QUEUES for this process (0: the environment's; HIP's default is 4, so with more "
                         "streams than queues two streams share one and a kernel can wait behind the other's)")
    ap.add_argument("--no-prof-timed", action="store_true",
                    help="time the headline steps without the per-kernel HIP events; the kernel table then comes "
                         "from a profiled pass of the same steps right after")
    ap.add_argument("--config3-steps", type=int, default=10,
                    help="also time BASELINE config 3 (TUM 640x480, 2000 feats, GF 160; 0: skip)")
    ap.add_argument("--config3-batch", type=int, default=1024)
    ap.add_argument("--kernel-times", choices=("rocprof", "events"), default="rocprof",
                    help="source of the per-kernel table: a rocprofv3 kernel trace of the same steps in a child "
                         "process (default, one GPU, not under a profiler) or the HIP events of the timed region")
    ap.add_argument("--kernel-trace-dir", default=None,
                    help="keep the rocprofv3 child's files (kernel trace, --stats summary, the timed region's "
                         "kernel_stats_timed.csv) in this directory")
    ap.add_argument("--enqueue", choices=("step", "split", "ring"), default="step",
                    help="host launch order of a step over the stream groups: each group's whole step in turn "
                         "(step), every group's extraction before any tracking (split, pipeline.step_all), or "
                         "group g's extraction before g - 1's tracking (ring, pipeline.GatedRing)")
    ap.add_argument("--dist-transport", choices=("rccl", "host"), default="rccl",
                    help="start-up exchange of --gpus N > 1: RCCL, one GPU per rank (the product path), or "
                         "host-staged collectives over a gloo group with the ranks sharing the visible GPUs "
                         "round-robin (a rehearsal of the N-rank bench path on one GPU)")
    ap.add_argument("--time-log", default=None,
                    help="file for Tracking::SaveTimeLog's per-frame stage log of stream 0 (default "
                         "gpurun_out/time_log.txt); the medians over all streams go to the record")
    ap.add_argument("--time-log-steps", type=int, default=12,
                    help="steps run with the stage log on after the timed region (0: skip)")
    ap.add_argument("--kernels-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--detail-out", default=None,
                    help="file for the full measurement record (per-kernel tables, legs); the stdout line is the "
                         "compact contract line (<= 8 KB) and names this file (default gpurun_out/bench_detail.json)")
    ap.add_argument("--no-reloc", action="store_true",
                    help="no keyframe databases: a lost stream stays LOST (the step then skips the BoW / candidate "
                         "launches); default: every stream relocalises against its scene's keyframes")
    args = ap.parse_args()

    if args.hw_queues > 0:  # before anything initialises the HIP runtime
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(args.hw_queues, 32))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # launch one process per GPU before anything touches the GPU
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
               "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    host_tp = args.dist_transport == "host"
    if world != args.gpus:
        raise SystemExit(f"WORLD_SIZE={world} does not match --gpus {args.gpus}")
    ktab, kqueues, knote = None, None, "HIP events (--kernel-times events)"
    if args.kernel_times == "rocprof" and not args.kernels_child:
        if world > 1:
            knote = "HIP events (rocprofv3 child only at one GPU)"
        elif _under_profiler():
            knote = "HIP events (this run is itself under a profiler)"
        else:  # a child process, started before this one touches the GPU
            ktab, kqueues, knote = rocprof_kernel_table(args)
            knote = knote or "rocprofv3 kernel trace of the same steps (child process)"

    import torch
    import torch.distributed as dist

    # the device of this rank: one per rank (RCCL), or shared round-robin by the
    # host-staged rehearsal of the N-rank path on fewer GPUs
    ndev = torch.cuda.device_count()
    local = local % ndev if host_tp else local
    torch.cuda.set_device(local)
    if world > 1:
        if host_tp:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    red_dev = "cpu" if host_tp else "cuda"  # tensors of the timing collectives

    from gf_orb_slam_amd import scene, synth
    from gf_orb_slam_amd.bow import ORBVocabulary
    from gf_orb_slam_amd.dist import GfDist, checksum, share_world
    from gf_orb_slam_amd.orb import Context
    from gf_orb_slam_amd.pipeline import CK, STATS, TR, FrontEnd, KeyframeDB, chain_extraction, GatedRing, step_all

    cam = args.camera
    refmap = not args.fixed_map
    if args.map is None:
        args.map = 2000 if args.fixed_map else 2100
    if args.stale_desc is None:
        args.stale_desc = 0.93 if args.fixed_map else 0.82
    B, G = args.batch, max(1, args.groups)
    if B % G:
        raise SystemExit(f"--batch {B} must be a multiple of --groups {G}")
    Bg = B // G
    S = min(args.scenes, B)

    # ---- start-up exchange (config 5): world, vocabulary, maps from rank 0 over RCCL
    t_su = time.perf_counter()
    ctx0 = Context(local)
    with _StdoutToStderr():
        gd = GfDist(ctx0, rank, world, transport=args.dist_transport)
    gd_world = gd.info()[1]
    scenes, maps, world_ck, world_span, world_bytes = share_world(
        gd, rank, lambda: build_world(cam, B, S, args.period, args.nfeatures, args.map, local, args.stale_desc,
                                      refmap, args.keyframes))
    voc = ORBVocabulary(synth.synth_vocabulary_fast(seed=7, k=10, L=6), ctx=ctx0) if rank == 0 else None
    voc = gd.bcast_vocab(voc, 0)
    voc_ck = voc.checksum()
    voc_span = gd.gather_ints([voc_ck])
    # Relocalisation's keyframe databases: KeyFrame::ComputeBoW of every keyframe
    # with the broadcast vocabulary (one database per scene, shared by its streams)
    dbs = None
    if refmap and not args.no_reloc:
        dbs = [KeyframeDB(m[3], m[4], voc.transform) for m in maps]
    W = scene.Workload(cam, B, n_scenes=S, period=args.period, seed=0, scenes=scenes, phase_offset=3 * rank)
    # (scene, phase) pairs of one step: with S * period >= B every sequence of
    # the step tracks a different frame (no group re-reads another's inputs)
    distinct = len(set(zip(W.scene_of.tolist(), W.phase.tolist())))
    frames = W.render_all(f"cuda:{local}").contiguous()
    T, V = W.boot_state()
    fes = []
    map_cks = []
    for g in range(G):
        sl = slice(g * Bg, (g + 1) * Bg)
        fe = FrontEnd(cam, args.nfeatures, Bg, args.map, args.gf_budget, ctx=Context(local))
        if rank == 0:
            for b in range(Bg):
                fe.set_map(b, *maps[W.scene_of[g * Bg + b]][:2])
        gd.bcast_map(fe, 0)  # every rank's streams get rank 0's maps, device to device
        for b in range(Bg):  # keyframe graphs: host-side, from the world blob
            load_map(fe, b, maps[W.scene_of[g * Bg + b]], with_points=False)
        map_cks.append(checksum(fe.read("map")) ^ checksum(fe.read("map_desc")))
        if dbs is not None:
            fe.set_vocab(voc)
            for b in range(Bg):
                fe.set_kfdb(b, dbs[W.scene_of[g * Bg + b]])
        for b in range(Bg):
            fe.set_rng(b, 1 + rank * B + g * Bg + b)
        fe.set_source(frames, W.scene_of[sl], W.phase[sl])
        fe.bootstrap(T[sl], V[sl], 0.0)
        fes.append(fe)
    gates = [] if args.no_gate else chain_extraction(fes)
    if args.gate_stage is not None and gates:
        for fe in fes:
            fe.set_gate_stage(args.gate_stage)
    if args.track_priority and G > 1:
        for fe in fes:
            fe.set_track_priority(-100)  # the device's most urgent priority
    map_span = gd.gather_ints(map_cks)
    torch.cuda.synchronize()
    t_su = time.perf_counter() - t_su
    startup = {"world_bytes": world_bytes, "vocabulary_nodes": voc.info()["nnodes"],
               "checksums_equal_across_ranks": bool(np.all(world_span[0] == world_span[1]) and
                                                    np.all(voc_span[0] == voc_span[1]) and
                                                    np.all(map_span[0] == map_span[1])),
               "world_checksum": world_ck, "vocabulary_checksum": voc_ck, "seconds": round(t_su, 2),
               "transport": ("RCCL" if not host_tp else "host-staged over gloo")
                            + " (gf_dist_bcast / gf_dist_bcast_vocab / gf_dist_bcast_map)"}

    # ---- warm-up
    hist = np.zeros(6, np.int64)
    lost = 0
    ring = GatedRing(fes) if args.enqueue == "ring" else None
    for _ in range(args.warmup):
        if ring is not None:
            ring.step()
            ring.finish()
        elif args.enqueue == "split":
            step_all(fes)
        else:
            for fe in fes:
                fe.step()
        for fe in fes:
            st = fe.read("stats")
            hist += np.bincount(st[STATS.index("branch")], minlength=6)[:6]
            lost += int((st[STATS.index("flags")] & 4 != 0).sum())
    for fe in fes:
        fe.sync()
        fe.write("hist", np.zeros((fe.B, 8), np.int32))  # running counters of the timed region
        fe.prof_enable(not args.no_prof_timed)  # per-launch HIP events (dispatch timestamps, GF_LAUNCH)
        fe.prof_reset()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_call = np.zeros((args.steps, G))  # host seconds inside each gf_frontend_step (enqueue only)
    t0 = time.perf_counter()
    for k in range(args.steps):
        if args.enqueue == "split":
            for g, fe in enumerate(fes):
                tc = time.perf_counter()
                fe.step_extract()
                t_call[k, g] = time.perf_counter() - tc
            for g, fe in enumerate(fes):
                tc = time.perf_counter()
                fe.step_track()
                t_call[k, g] += time.perf_counter() - tc
        elif args.enqueue == "ring":
            tc = time.perf_counter()
            ring.step()
            t_call[k, :] = (time.perf_counter() - tc) / G
        else:
            for g, fe in enumerate(fes):
                tc = time.perf_counter()
                fe.step()
                t_call[k, g] = time.perf_counter() - tc
    if ring is not None:
        ring.finish()
    t_enq = time.perf_counter() - t0
    for fe in fes:
        fe.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    dt_rank = dt
    tt = torch.tensor([dt], dtype=torch.float64, device=red_dev)
    if world > 1:
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    dt = float(tt.item())
    # every rank's own wall time of the timed steps (the straggler shows here)
    rank_dt = torch.zeros(world, dtype=torch.float64, device=red_dev)
    rank_dt[rank] = dt_rank
    if world > 1:
        dist.all_reduce(rank_dt, op=dist.ReduceOp.SUM)
    rank_dt = rank_dt.cpu().numpy()
    if args.kernels_child:  # the profiled child ends with the timed region
        print(json.dumps({"kernels_child": True, "ms_per_step": round(dt / args.steps * 1e3, 3)}))
        for fe in fes:
            fe.close()
        return
    stats = [fe.stats() for fe in fes]
    final = {k: np.concatenate([s[k] for s in stats]) for k in STATS}
    thist = np.concatenate([fe.read("hist") for fe in fes]).astype(np.int64)  # [B][8] over the timed steps
    trk = np.concatenate([fe.read("track") for fe in fes])  # GF_FE_TRACK after the timed steps
    if args.no_prof_timed:  # the kernel table from a profiled pass of the same steps
        for fe in fes:
            fe.prof_enable(True)
        for _ in range(args.steps):
            for fe in fes:
                fe.step()
        for fe in fes:
            fe.sync()
    prof = {}
    for fe in fes:
        for k, (ms, cnt) in fe.prof_report().items():
            a = prof.setdefault(k, [0.0, 0])
            a[0] += ms
            a[1] += cnt
        fe.prof_enable(False)
    mix = thist[:, :6].sum(0)
    ldets_total = float(thist[:, 6].sum())
    local_total = float(thist[:, 7].sum())

    frames_total = world * B * args.steps
    fps = frames_total / dt
    kb = kernel_bytes(cam, args.nfeatures)
    iters = np.stack([final["iter1"], final["iter2"]]).astype(np.float64)
    nedges = np.stack([final["edges1"], final["edges2"]]).astype(np.float64)
    # SURVEY §8d units of work per launch (one launch = one group of Bg streams)
    work = {"k_pyramid": ("hbm", kb["k_pyramid"] * Bg, "pyramid levels 1.. of %d frames in one launch: level 0 read + levels 1.. written (P)" % Bg),
            "k_blur_fast": ("hbm", kb["k_blur_fast"] * Bg,
                            "%d frames x 3 P bytes (level read, blurred level + FAST score map written)" % Bg),
            "k_describe": ("hbm", kb["k_describe"] * Bg, "%d frames x 60 N bytes" % Bg)}
    if "k_active_match" in prof:
        n_am = prof["k_active_match"][1]
        work["k_active_match"] = ("hbm", 224.0 * ldets_total * world / max(world * n_am, 1),
                                  "224 B x logDet evaluations (E_ld, %.0f per frame in the timed region)"
                                  % (ldets_total / max(B * args.steps, 1)))
    if "k_pose_opt" in prof:
        # edges x LM iterations of the last timed step (both PoseOptimization calls), per launch
        ei = float((nedges * iters).sum()) / (2 * G)
        work["k_pose_opt"] = ("f64", 160.0 * ei, "160 flop x edges x LM iterations (%.0f edge-iterations per "
                                                  "launch, last timed step)" % ei)
    # matchers (SURVEY §8d B_match = 48 M + 36 C + 8 N per frame, C = area
    # candidates counted on the device, GF_ST_CAND_*), from the last timed step
    nkp_last = np.concatenate([fe.read("nkp") for fe in fes]).astype(np.float64)
    m2_q = np.where(final["branch"] == 2, final["nlocal"] if refmap else args.map, 0).astype(np.float64)
    b_m3 = 48.0 * nkp_last + 36.0 * final["cand_last"] + 8.0 * nkp_last
    b_proj = 48.0 * (m2_q + final["nleft"]) + 36.0 * final["cand_proj"] + 2 * 8.0 * nkp_last
    if "k_match_lastframe" in prof:
        work["k_match_lastframe"] = ("hbm", float(b_m3.sum()) / G,
                                     "48 M + 36 C + 8 N per frame: SearchByProjection(Cur, Last), M = last-frame "
                                     "keypoints, C = %.0f area candidates per frame (device-counted), last timed step"
                                     % float(final["cand_last"].mean()))
    if "k_match_project" in prof:
        work["k_match_project"] = ("hbm", float(b_proj.sum()) / (2 * G),
                                   "48 M + 36 C + 8 N per frame over SearchByProjection(F, local) and "
                                   "SearchByProjection_Budget (two launches per step), C = %.0f area candidates per "
                                   "frame, last timed step" % float(final["cand_proj"].mean()))
    PEAK = {"hbm": (8000.0, "GB/s"), "f64": (78.6, "TFLOP/s")}

    def price(k, ms_avg, traffic=None):
        kind, units, what = work[k]
        s_ = ms_avg / 1e3
        ach = units / s_ / (1e9 if kind == "hbm" else 1e12)
        peak, unit = PEAK[kind]
        return {"kernel": k, "bound": "hbm" if kind == "hbm" else "mfma", "achieved": round(ach, 4), "peak": peak,
                "unit": unit, "frac": round(ach / peak, 6), "traffic": traffic,
                ("algorithmic_bytes_per_launch" if kind == "hbm" else "algorithmic_flops_per_launch"): units,
                "work": what, "avg_launch_ms": round(ms_avg, 4), "launches": prof[k][1]}

    # the rocprof dispatch durations of the same steps (child process), per
    # launch of each priced kernel's HIP-event scope: DESIGN §5 takes them as
    # the honest per-kernel times (HIP events also count queue waits behind
    # other streams' kernels), so every `frac` is priced from them when present
    rp = {k: (sum(v) / 1e6, len(v)) for k, v in ktab.items()} if ktab else None
    SCOPE = {"k_active_match": ["k_active_match", "k_active_match_overflow"],
             "k_match_lastframe": ["k_match_seq", "k_match_seq_pre"], "k_match_project": ["k_match"],
             "k_pose_opt": ["k_pose_opt_frames"], "k_select": ["k_select_cells", "k_select_level"],
             "k_fast_cells": ["k_fast_cells", "k_fast_cells_band"]}

    def rp_total(k):
        return sum(rp[n][0] for n in SCOPE.get(k, [k]) if n in rp) if rp else 0.0

    if rp:
        priced = {}
        for k in work:
            if k in prof and rp_total(k) > 0:
                ev = prof[k][0] / prof[k][1]
                if k == "k_active_match" and "k_active_match_overflow" in prof:
                    ev = (prof[k][0] + prof["k_active_match_overflow"][0]) / prof[k][1]
                if k == "k_match_lastframe" and "k_match_seq_pre" in prof:
                    ev = (prof[k][0] + prof["k_match_seq_pre"][0]) / prof[k][1]
                priced[k] = price(k, rp_total(k) / prof[k][1])
                priced[k].update({"timing": "rocprof", "avg_launch_ms_events": round(ev, 4),
                                  "events_over_rocprof": round(ev / (rp_total(k) / prof[k][1]), 3),
                                  "rocprof_kernels": SCOPE.get(k, [k])})
            elif k in prof:  # no rocprof dispatch under this scope's names: HIP events, said so
                ev = prof[k][0]
                for extra in {"k_active_match": "k_active_match_overflow",
                              "k_match_lastframe": "k_match_seq_pre"}.get(k, "").split():
                    ev += prof.get(extra, (0.0, 0))[0]
                priced[k] = price(k, ev / prof[k][1])
                priced[k]["timing"] = "hip_events (no rocprof scope)"
    else:
        priced = {k: price(k, prof[k][0] / prof[k][1]) for k in work if k in prof}
        for k in priced:
            priced[k]["timing"] = "hip_events"
    if rp is None and "k_active_match" in priced and "k_active_match_overflow" in prof:
        # two-pass launch (gf.hip obs_active_match): the log-dets counted per
        # frame include the frames the overflow pass redid, so the rate is
        # priced over both passes' time per launch pair
        ms_pair = (prof["k_active_match"][0] + prof["k_active_match_overflow"][0]) / prof["k_active_match"][1]
        first = priced["k_active_match"]["avg_launch_ms"]
        priced["k_active_match"] = price("k_active_match", ms_pair)
        priced["k_active_match"].update({
            "avg_launch_ms_first_pass": first,
            "avg_launch_ms_overflow_pass": round(prof["k_active_match_overflow"][0]
                                                 / max(prof["k_active_match_overflow"][1], 1), 4),
            "timing_note": "avg_launch_ms = small-pool pass + overflow pass (k_active_match_overflow) per step "
                           "and group; rocprof lists them as two kernels"})
    if "k_describe" in priced:
        # §8d prices describe at its outputs; the stage must also read the
        # level and the blurred level around every keypoint: the planes once
        bp = kb["k_describe_planes"] * Bg
        ms_d = priced["k_describe"]["avg_launch_ms"]
        priced["k_describe"]["with_planes_read"] = {
            "algorithmic_bytes_per_launch": bp, "achieved": round(bp / (ms_d / 1e3) / 1e9, 2), "unit": "GB/s",
            "frac": round(bp / (ms_d / 1e3) / 1e9 / 8000.0, 6),
            "work": "%d frames x (2 P + 60 N): the IC_Angle level and the rBRIEF blurred level read once" % Bg}
    if rp is None and "k_match_lastframe" in priced and "k_match_seq_pre" in prof:
        # the per-query precompute and the ordered pass are one SearchByProjection(Cur, Last)
        ms_pair = (prof["k_match_lastframe"][0] + prof["k_match_seq_pre"][0]) / prof["k_match_lastframe"][1]
        priced["k_match_lastframe"] = price("k_match_lastframe", ms_pair)
        priced["k_match_lastframe"]["timing_note"] = "avg_launch_ms = k_match_seq_pre + k_match_seq per launch"
    for k in priced:
        if work[k][0] == "f64":
            priced[k]["peak_note"] = "FP64 peak (AMD spec, vector = matrix on MI355X); this kernel is f64 VALU"
    if rp:
        top = max(rp, key=lambda k: rp[k][0])
        dom = max(priced, key=rp_total) if priced else None
    else:
        top = max(prof, key=lambda k: prof[k][0])
        dom = max(priced, key=lambda k: prof[k][0])
    traffic_src = None
    for cand in ("r06",):  # PMC traffic measured on this round's build and workload only
        try:
            pmc = json.load(open(os.path.join(ROOT, "profiles", cand, "pmc_traffic.json")))
            if pmc.get("batch") == Bg:
                pk = pmc.get("kernels", {})
                for k in priced:  # every priced kernel whose dispatches the PMC table holds
                    names = [n for n in SCOPE.get(k, [k]) if n in pk]
                    if names:
                        priced[k]["traffic"] = round(sum(pk[n]["traffic_bytes"] for n in names))
                        priced[k]["traffic_min"] = round(sum(pk[n].get("traffic_bytes_min", pk[n]["traffic_bytes"])
                                                             for n in names))
                traffic_src = (f"profiles/{cand}/pmc_traffic.json: traffic = 2 x FETCH_SIZE + WRITE_SIZE per launch "
                               "(exact for 128-B read requests), traffic_min = FETCH_SIZE + WRITE_SIZE (scattered "
                               "64-B requests; calibration in that file)")
                break
        except (OSError, ValueError, KeyError):
            pass
    if dom is None:
        raise RuntimeError("no SURVEY §8d kernel was timed in the step (empty kernel table)")
    roof = dict(priced[dom])
    roof["traffic_source"] = traffic_src
    roof["frames_per_launch"] = Bg
    roof["dominant_by"] = ("total rocprof dispatch time" if rp else "total HIP-event time") + \
        " over the timed region among the SURVEY §8d-priced kernels"
    tab = rp if rp else {k: tuple(v) for k, v in prof.items()}
    if top not in SCOPE.get(dom, [dom]):
        roof["largest_kernel"] = {"kernel": top, "avg_launch_ms": round(tab[top][0] / tab[top][1], 4)}
    roof["other_kernels"] = {k: v for k, v in priced.items() if k != dom}
    ext_ms = sum(tab[n][0] for k in ("k_pyramid", "k_blur_fast", "k_fast_cells", "k_select", "k_describe")
                 for n in (SCOPE.get(k, [k]) if rp else [k]) if n in tab)
    ext_bw = kb["extract_total"] * B * args.steps / (ext_ms / 1e3) / 1e9 if ext_ms else None
    gf_kernels = [k for k in tab if k.startswith(("k_obs", "k_onepoint", "k_active"))]
    gf_ms = sum(tab[k][0] for k in gf_kernels)
    all_ms = sum(v[0] for v in tab.values())
    pose_ms = prof.get("k_pose_opt", (0.0, 1))
    pose_avg_ms = pose_ms[0] / max(pose_ms[1], 1)
    mean_iters = float(iters.mean())
    nfr = max(B * args.steps, 1)
    local_mean = float(final["nlocal"].mean()) if refmap else float(args.map)

    out = {
        "metric": "front-end fps (extract+match+GF-select) @ 752x480/1000 feats; pose-opt ms/iter",
        "value": round(fps, 2),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8/int32 (extract, match), f64 (GF, pose LM)",
        "data": "synthetic: rendered sequences (textured-plane rooms, closed EuRoC-speed loops), %s with %.0f%% "
                "stale (random) map descriptors; no dataset reachable"
                % ("keyframe maps (%d keyframes of a mapping sweep, covisibility graph)" % args.keyframes if refmap
                   else "keyframe-built fixed local maps", 100 * args.stale_desc),
        "config": {"workload": f"config 2: {cam} {W.cam[0]}x{W.cam[1]}, {args.nfeatures} feats, GF budget "
                               f"{args.gf_budget}, "
                               + (f"{args.keyframes}-keyframe maps of {args.map} points, the local map (~"
                                  f"{local_mean:.0f} points) rebuilt every frame by Tracking::UpdateReference"
                                  if refmap else f"{args.map}-point fixed local maps")
                               + f" ({args.stale_desc:.2f} stale descriptors: ~60 motion-model matches, "
                               f"runActiveMapMatching every frame), {B} "
                               f"tracked sequences per GPU in {G} groups; step = one frame of every sequence "
                               f"through Tracking::GrabImage (WORKING): extract, motion model + "
                               f"SearchByProjection(last) + PoseOptimization, "
                               + ("UpdateReference (local keyframes + local points), " if refmap else "")
                               + f"GF SearchReferencePointsInFrustum "
                               f"(FRAME_INFO, isInFrustum, MAP_INFO, runActiveMapMatching), PoseOptimization, "
                               f"motion update, next-frame MAP_INFO prediction, SearchAdditionalMatchesInFrame",
                   "sequences_per_gpu": B, "stream_groups": G, "update_reference": refmap,
                   "extraction_gate": bool(gates), "enqueue": args.enqueue,
                   "tracking_stream_priority": bool(args.track_priority and G > 1),
                   "parallelism": f"{B} sequences x {world} ranks (one process per GPU)"
                                  if not host_tp else
                                  f"{B} sequences x {world} ranks on {min(world, ndev)} GPU(s) "
                                  f"(host-staged rehearsal of the N-rank path)",
                   "distinct_frames_per_step": distinct},
        "startup": startup,
        "ranks": {"world": world, "communicator_world": gd_world, "transport": args.dist_transport,
                  "devices_used": min(world, ndev) if host_tp else world,
                  "frames_per_s": [round(B * args.steps / float(x), 1) for x in rank_dt],
                  "ms_per_step": [round(float(x) / args.steps * 1e3, 3) for x in rank_dt],
                  "min_frames_per_s": round(B * args.steps / float(rank_dt.max()), 1),
                  "max_frames_per_s": round(B * args.steps / float(rank_dt.min()), 1),
                  "max_over_min_ms": round(float(rank_dt.max() / rank_dt.min()), 4),
                  "note": "each rank's own wall time of the timed steps; `value` uses the max over ranks"},
        "host_enqueue": {"ms_per_step": round(t_enq / args.steps * 1e3, 3),
                         "call_ms_avg": [round(float(x) * 1e3, 3) for x in t_call.mean(axis=0)],
                         "call_ms_max": round(float(t_call.max()) * 1e3, 3),
                         "note": "host time inside gf_frontend_step per group (launches only): close to "
                                 "ms_per_step means the host, not the GPU, paces the steps"},
        "roofline": roof,
        "pose_opt": {"ms_per_iter": round(pose_avg_ms / max(mean_iters, 1e-9), 5),
                     "avg_launch_ms": round(pose_avg_ms, 4), "mean_iterations": round(mean_iters, 2),
                     "mean_edges": [round(float(x), 1) for x in nedges.mean(axis=1)],
                     "note": f"ms_per_iter = launch time / mean LM iterations ({Bg} problems per launch run "
                             f"concurrently)"},
        "gf_select": {"kernels": gf_kernels, "ms_per_step": round(gf_ms / args.steps, 4),
                      "share_of_kernel_time": round(gf_ms / all_ms, 4) if all_ms else None,
                      "logdets_per_frame": round(ldets_total / nfr, 1),
                      "active_matches_per_frame": round(local_total / nfr, 2),
                      "note": ("rocprof dispatch" if rp else "HIP-event") + " time of the GF kernels (FRAME_INFO / "
                              "MAP_INFO builds, one-point precompute, runActiveMapMatching) over all kernel time; "
                              "groups overlap"},
        "tracking": {"branch_mix_timed": {"leftovers_only": int(mix[1]), "search_by_projection": int(mix[2]),
                                          "active_matching": int(mix[3]), "nothing_in_view": int(mix[4]),
                                          "budget_cut": int(mix[5])},
                     "branch_mix_warmup": {"leftovers_only": int(hist[1]), "search_by_projection": int(hist[2]),
                                           "active_matching": int(hist[3]), "nothing_in_view": int(hist[4])},
                     "keyframe_databases": dbs is not None,
                     "streams_lost_at_end": int((trk[:, TR["state"]] == 1).sum()),
                     "last_step_paths": {p: int((trk[:, TR["path"]] == i).sum()) for i, p in
                                         enumerate(["motion_model", "previous_frame_fallback", "previous_frame",
                                                    "relocalisation"])},
                     "mean_local_map_points": round(local_mean, 1),
                     "mean_inliers": round(float(final["inl2"].mean()), 1),
                     "mean_last_frame_matches": round(float(final["m3"].mean()), 1),
                     "mean_num_to_match": round(float(final["to_match"].mean()), 1),
                     "mean_in_view": round(float(final["in_view"].mean()), 1),
                     "mean_additional_matches": round(float(final["extra"].mean()), 1),
                     "lost_frames_warmup": lost,
                     "lost_frames_last_step": int((final["flags"] & 4 != 0).sum())},
        "extraction_stage": {"ms_per_frame": round(ext_ms / (B * args.steps), 5),
                             "algorithmic_GBps": round(ext_bw, 2) if ext_bw else None},
        "kernels_note": f"{knote}: per dispatch over the timed region; each launch covers one group ({Bg} "
                        f"sequences) and the {G} groups' launches overlap (extraction stages chained one group at a "
                        f"time when extraction_gate), so ms_per_step sums exceed the wall time per step"
                        + (f"; the child's timed region used {kqueues} hardware queues" if kqueues else ""),
        "kernels": {k: {"avg_ms": round(v[0] / max(v[1], 1), 4), "launches": v[1],
                        "ms_per_step": round(v[0] / args.steps, 4)} for k, v in sorted(tab.items(),
                                                                                     key=lambda kv: -kv[1][0])},
    }
    if rp:  # the HIP-event scopes of this run (they include queue waits behind other streams' kernels)
        out["kernels_hip_events"] = {k: {"avg_ms": round(v[0] / max(v[1], 1), 4), "launches": v[1]}
                                     for k, v in prof.items()}
    if args.isolated_steps > 0:
        # the priced kernel with one group running alone (after the timed
        # region): in the timed region the other groups' tracking kernels share
        # its CUs, so its HIP-event duration there includes that contention
        fe = fes[0]
        fe.prof_enable(True)
        fe.prof_reset()
        for _ in range(args.isolated_steps):
            fe.step()
        fe.sync()
        rep = fe.prof_report()
        fe.prof_enable(False)
        iso = {}
        for k in priced:
            if k in rep:
                e = price(k, rep[k][0] / rep[k][1])
                iso[k] = {"avg_launch_ms": e["avg_launch_ms"], "achieved": e["achieved"], "frac": e["frac"]}
        out["roofline"]["isolated"] = {**iso.get(dom, {}), "steps": args.isolated_steps,
                                       "others": {k: v for k, v in iso.items() if k != dom},
                                       "note": "one group alone, HIP events; `frac` above is the timed region "
                                               "with the groups overlapping"}
    if args.budget_steps > 0:
        # the reference's own time budgets (SURVEY §7 budgets-on leg): time_total_match = 15 ms
        # (Tracking.cc:3230) and the post-publish rest 1 / (0.5 fps) - 2 ms (Tracking.cc:866),
        # measured on the device clock from each step's start
        sel_s = 1.0 / (0.5 * 20.0) - 0.002
        for fe in fes:
            fe.set_budgets(0.015, sel_s)
            fe.write("hist", np.zeros((fe.B, 8), np.int32))
        for fe in fes:  # the first budgeted step runs eagerly
            fe.step()
        for fe in fes:
            fe.sync()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        cut_f = cut_s = 0
        for _ in range(args.budget_steps):
            for fe in fes:
                fe.step()
        for fe in fes:
            fe.sync()
        db = time.perf_counter() - t1
        caps = {"isInFrustum": 32, "map_info": 64, "active_matching": 128, "no_time_left": 16,
                "map_info_next": 256, "visibility_pass": 512, "budget_matcher": 1024}
        last = {k: 0 for k in caps}
        sofar = []
        for fe in fes:
            st = fe.read("stats")
            for k, bit in caps.items():
                last[k] += int((st[STATS.index("flags")] & bit != 0).sum())
            sofar.append(fe.read("clock")[:, CK["sofar"]])
            fe.set_budgets()
        bh = np.concatenate([fe.read("hist") for fe in fes]).astype(np.int64)
        sofar = np.concatenate(sofar) / 1e8
        out["budgets_on"] = {"match_s": 0.015, "select_s": round(sel_s, 4), "steps": args.budget_steps,
                             "frames_per_s": round(B * args.budget_steps / db, 1),
                             "ms_per_step": round(db / args.budget_steps * 1e3, 3),
                             "branch_mix": {"active_matching": int(bh[:, 3].sum()),
                                            "leftovers_only": int(bh[:, 1].sum())},
                             "frames_cut": int(bh[:, 5].sum()), "frames": int(B * (args.budget_steps + 1)),
                             "last_step_caps": last,
                             "timeCost_sofar_ms": {"median": round(float(np.median(sofar)) * 1e3, 3),
                                                   "max": round(float(sofar.max()) * 1e3, 3)},
                             "note": "gf_set_budgets with the reference's budgets (abi.h: each cap's timer where "
                                     "the reference starts it, frame clock after the extraction gate); parity "
                                     "mode (+inf) is the headline"}
    if args.time_log_steps > 0:
        # Tracking::SaveTimeLog's per-frame stage log (gf_frontend_set_time_log),
        # after the timed region: device-clock stage boundaries of every group
        from gf_orb_slam_amd.pipeline import TIME_LOG_COLUMNS
        for fe in fes:
            fe.set_time_log(args.time_log_steps)
        for _ in range(args.time_log_steps):
            for fe in fes:
                fe.step()
        logs = [fe.time_log() for fe in fes]
        tl_file = args.time_log or os.path.join(ROOT, "gpurun_out", "time_log.txt")
        try:
            os.makedirs(os.path.dirname(os.path.abspath(tl_file)), exist_ok=True)
            fes[0].save_time_log(tl_file, 0)
        except OSError as e:
            tl_file = f"(not written: {e})"
        med = {}
        for c in TIME_LOG_COLUMNS[1:]:
            v = np.concatenate([lg[c].reshape(-1) for lg in logs]).astype(np.float64)
            med[c] = round(float(np.median(v)) * (1e3 if c.startswith("time_") else 1.0), 4)
        out["time_log"] = {"file": os.path.relpath(tl_file, ROOT) if os.path.isabs(tl_file) else tl_file,
                           "steps": args.time_log_steps, "streams": B, "median": med,
                           "unit": "ms (time_*), landmarks (lmk_*)",
                           "note": "Tracking::SaveTimeLog columns (Tracking.h:254-280) per frame and stream; stage "
                                   "boundaries on the device clock, shared by the streams of a group (batched "
                                   "stages), counts per stream; the groups overlap, so a stage's time includes "
                                   "the other groups' kernels beside it"}
        for fe in fes:
            fe.set_time_log(0)
    for fe in fes:
        fe.close()
    if rank == 0 and args.single_stream_steps > 0:
        # one sequence alone: per-frame latency, the step replayed as one HIP graph
        fe = FrontEnd(cam, args.nfeatures, 1, args.map, args.gf_budget, ctx=Context(local))
        load_map(fe, 0, maps[W.scene_of[0]])
        fe.set_rng(0, 1)
        fe.set_source(frames, W.scene_of[:1], W.phase[:1])
        fe.bootstrap(T[:1], V[:1], 0.0)
        res = {}
        for mode in ("eager", "graph"):
            for _ in range(3):
                fe.step()
            if mode == "graph":
                fe.capture_graph()
            fe.sync()
            t1 = time.perf_counter()
            for _ in range(args.single_stream_steps):
                fe.step()
            fe.sync()
            d = (time.perf_counter() - t1) / args.single_stream_steps
            res[mode] = {"ms_per_frame": round(d * 1e3, 3), "fps": round(1.0 / d, 1)}
        best = min(res, key=lambda m: res[m]["ms_per_frame"])  # both launch modes measured; the faster one leads
        out["single_stream"] = {**res[best], "mode": best, "graph": res["graph"], "eager": res["eager"],
                                "steps": args.single_stream_steps}
        fe.close()
    if rank == 0 and args.pcie_steps > 0:
        # frames handed over from host memory: the PCIe copy inside the step (not `value`)
        fe = FrontEnd(cam, args.nfeatures, Bg, args.map, args.gf_budget, ctx=Context(local))
        for b in range(Bg):
            load_map(fe, b, maps[W.scene_of[b]])
        fe.set_source(frames, W.scene_of[:Bg], W.phase[:Bg])
        fe.bootstrap(T[:Bg], V[:Bg], 0.0)
        fh = frames.cpu().numpy()
        host = [np.stack([fh[W.scene_of[b], (W.phase[b] + k) % W.period] for b in range(Bg)])
                for k in range(1, args.pcie_steps + 2)]
        fe.step_host(host[0])
        fe.sync()
        t1 = time.perf_counter()
        for k in range(args.pcie_steps):
            fe.step_host(host[k + 1])
        fe.sync()
        d = (time.perf_counter() - t1) / args.pcie_steps
        out["pcie_inclusive"] = {"frames_per_s": round(Bg / d, 1), "ms_per_step": round(d * 1e3, 3),
                                 "sequences": Bg, "note": "one group, frames copied from pageable host memory "
                                                          "in each step (hipMemcpyAsync), not the headline value"}
        fe.close()
    if rank == 0 and args.lba_batch > 0:
        out["local_ba"] = lba_leg(args.lba_batch, cpu=not args.no_cpu_baseline)
    if rank == 0 and world == 1 and args.config3_steps > 0:
        out["config3"] = config3_leg(local, args.config3_batch, G, args.config3_steps, 3)
    if rank == 0 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cam, args.nfeatures, args.map, args.gf_budget, 20.0, maps, W,
                                           frames.cpu().numpy(), budget_s=args.cpu_seconds)
        ac = out["cpu_baseline"]["all_cores"]
        phys = out["cpu_baseline"]["host"]["physical_cores"]
        out["cpu_baseline"]["vs_gpu"] = {
            "single_sequence_speedup": round(out.get("single_stream", {}).get("fps", 0) / out["cpu_baseline"]["value"],
                                             1) if "single_stream" in out else None,
            "aggregate_vs_one_core": round(fps / world / out["cpu_baseline"]["value"], 1),
            "aggregate_vs_all_cores": round(fps / world / ac["value"], 1),
            "all_cores_used": ac["cores"],
            "aggregate_vs_whole_host_linear": round(fps / world / (ac["value"] * phys / ac["cores"]), 1),
            "note": "aggregate = this GPU's frames/s; all_cores = every physical core of the job's CPU share, "
                    "pinned; whole_host_linear scales that figure linearly to all %d physical cores of the "
                    "node (an extrapolation, not a measurement)" % phys}
        # the reference's own published figure (~11-16 ms per
        # frame on EuRoC, one tracking thread): the speed-ups against it
        ss = out.get("single_stream", {}).get("fps")
        out["cpu_baseline"]["vs_published"] = {
            "published_ms_per_frame": [11.0, 16.0], "published_frames_per_s": [62.5, 90.9],
            "single_sequence_speedup": [round(ss / 90.9, 1), round(ss / 62.5, 1)] if ss else None,
            "aggregate_speedup_one_gpu": [round(fps / world / 90.9, 1), round(fps / world / 62.5, 1)],
            "note": "GPU figures over the reference's published per-frame latency range (read off its plot, "
                    "hardware not stated); `value` above is this repo's scalar C++ port timed here"}
    if rank == 0:
        detail = args.detail_out or os.path.join(ROOT, "gpurun_out", "bench_detail.json")
        try:
            os.makedirs(os.path.dirname(os.path.abspath(detail)), exist_ok=True)
            with open(detail, "w") as fh:
                json.dump(out, fh, indent=1)
        except OSError as e:
            detail = f"(not written: {e})"
        line = compact_line(out, os.path.relpath(detail, ROOT) if os.path.isabs(detail) else detail)
        print(line, flush=True)
    gd.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
