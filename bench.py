#!/usr/bin/env python3
"""GF-ORB-SLAM front-end benchmark (BASELINE.json metric).

Metric: front-end fps (extract + match + GF-select) @ 752x480 / 1000 feats,
plus pose-opt ms/iter (config 2: EuRoC-geometry synthetic frames, GF budget
100, one MI355X per rank). One step = one frame of each of B independent
streams through the device-resident hot path (gf_orb_slam_amd.pipeline.
FrontEnd: extract, motion-model matching, pose LM, GF active matching, pose
LM); value = frames of all ranks / wall time. Multi-GPU: one process per GPU (torchrun), streams shard across ranks
with no data-path collective ("weak" scaling); rank 0 broadcasts the shared
vocabulary/map blob over RCCL once before timing.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# Algorithmic bytes per frame for the extraction kernels,
# computed from the level sizes: P = sum of pyramid pixels.
LEVELS = {"euroc": [(752, 480), (627, 400), (522, 333), (435, 278), (363, 231), (302, 193), (252, 161), (210, 134)],
          "tum": [(640, 480), (533, 400), (444, 333), (370, 278), (309, 231), (257, 193), (214, 161), (179, 134)]}


def kernel_bytes(camera: str, nfeat: int) -> dict:
    px = [w * h for w, h in LEVELS[camera]]
    P, P0, P7 = sum(px), px[0], px[-1]
    return {
        "k_resize": (P - P7) + (P - P0),  # read level l-1, write level l
        "k_blur_fast": 3 * P,             # blur read + write every level, FAST reads every pixel once
        "k_describe": 60 * nfeat,         # 32 B descriptor + 28 B keypoint out
        "extract_total": (P - P7) + (P - P0) + P + 2 * P + 60 * nfeat,
    }


def _cpu_worker(args) -> tuple:
    """One host core running the oracle chain on its own stream (no GPU)."""
    camera, nfeat, stream, budget_s = args
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_chain

    from gf_orb_slam_amd import synth

    cam = synth.CAMERAS[camera]
    preps = [oracle_chain.prepare(camera, nfeat, synth.synth_frame(cam[0], cam[1], synth.frame_seed(stream, i)),
                                  1000 + 7 * stream + i) for i in range(2)]
    n, times, t0 = 0, [], time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        t1 = time.perf_counter()
        oracle_chain.step(preps[n % len(preps)])
        times.append(time.perf_counter() - t1)
        n += 1
    return n, time.perf_counter() - t0, times


def cpu_baseline(camera: str, nfeat: int, budget_s: float = 12.0, workers: int = 16) -> dict:
    """The oracle chain (CPU restatement) on a bounded sample of the same
    workload, one full front-end step per frame (tests/oracle_chain.py):
    (i) one core, one stream — the baseline value — with per-frame median and
    p90; (ii) `workers` host cores, one independent stream per process
    (throughput), as SURVEY.md §8(d) asks."""
    import multiprocessing as mp
    import platform

    n, dt, times = _cpu_worker((camera, nfeat, 99, budget_s))
    t = np.sort(np.asarray(times))
    out = {"value": round(n / dt, 3), "unit": "frames/s", "cores": 1, "kind": "port",
           "sample": f"{n} frames ({camera} {nfeat} feats, 2000-point local map, GF budget 100): extract + "
                     f"motion model + SearchByProjection(last) + PoseOptimization + G1-G7 active matching + "
                     f"PoseOptimization, 1 thread, {dt:.1f} s",
           "ms_per_frame_median": round(float(np.median(t)) * 1e3, 2),
           "ms_per_frame_p90": round(float(t[int(0.9 * (len(t) - 1))]) * 1e3, 2)}
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as fh:
            cpu_model = next((ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name")), "")
    except OSError:
        pass
    w = max(1, min(workers, os.cpu_count() or 1))
    ctx = mp.get_context("spawn")  # fresh interpreters: the workers never touch the GPU
    with ctx.Pool(w) as pool:
        res = pool.map(_cpu_worker, [(camera, nfeat, 200 + i, budget_s * 0.75) for i in range(w)])
    frames = sum(r[0] for r in res)
    wall = max(r[1] for r in res)
    out["all_cores"] = {"value": round(frames / wall, 2), "unit": "frames/s", "cores": w,
                        "sample": f"{frames} frames, one stream per process, {wall:.1f} s"}
    out["host"] = {"nproc": os.cpu_count(), "cpu_model": cpu_model or platform.processor()}
    return out


def single_stream(camera: str, nfeat: int, budget: int, steps: int) -> dict:
    """Per-frame latency of ONE sequence (B = 1) through the same device path."""
    import torch

    from gf_orb_slam_amd import synth
    from gf_orb_slam_amd.pipeline import FrontEnd

    w, h = synth.CAMERAS[camera][:2]
    fe = FrontEnd(camera, nfeat, 1, 2000, gf_budget=budget, seed=99)
    fe.load_frames(synth.synth_frame(w, h, synth.frame_seed(99, 0))[None])
    fe.build_maps()
    for _ in range(3):
        fe.step()
    fe.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fe.step()
    fe.sync()
    dt = (time.perf_counter() - t0) / steps
    return {"ms_per_frame": round(dt * 1e3, 3), "fps": round(1.0 / dt, 2), "steps": steps}


def schur_flops(prob: dict) -> float:
    """Algorithmic flops of one Schur contraction (k_ba_gemm) for one LBA
    window: per map point with k edges to local (free) keyframes, the k(k+1)/2
    6x6 blocks W_i Hpl_j^T (3 products each) and the k 6-vectors Hpl_i db."""
    free = prob["kf_kind"][prob["edge_kf"]] == 0
    k = np.bincount(prob["edge_pt"][free], minlength=len(prob["pt_pos"])).astype(np.float64)
    return float((k * (k + 1) / 2 * 36 * 3 * 2 + k * 6 * 3 * 2).sum())


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
            entry["schur_gemm"] = {"bound": "mfma", "achieved": round(tf, 4), "peak": 78.6, "unit": "TFLOP/s",
                                   "frac": round(tf / 78.6, 6), "algorithmic_flops_per_launch": flops,
                                   "note": "f64 MFMA 16x16x4; peak = AMD spec FP64 matrix (not measured here)"}
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


def share_startup_state(dist, device, world: int, rank: int, vocab_levels: int = 6):
    """The one exchange step: rank 0 builds the ORB
    vocabulary (ORBvoc-sized synthetic tree: k = 10, L = 6, 1.1 M nodes, 50 MB
    packed) and broadcasts it to every rank — RCCL over xGMI on the GPU node,
    gloo in the CPU tests. Returns (vocabulary dict, checksum); every rank must
    hold the same checksum."""
    import torch

    from gf_orb_slam_amd import synth

    size = torch.zeros(1, dtype=torch.int64, device=device)
    if rank == 0:
        blob_np = synth.pack_vocabulary(synth.synth_vocabulary_fast(seed=7, k=10, L=vocab_levels))
        size[0] = blob_np.size
    if world > 1:
        dist.broadcast(size, src=0)
    n = int(size.item())
    blob = torch.empty(n, dtype=torch.uint8, device=device)
    if rank == 0:
        blob.copy_(torch.from_numpy(blob_np))
    if world > 1:
        dist.broadcast(blob, src=0)
    host = blob.cpu().numpy()
    ck = int(host[:: max(1, n // 65536)].astype(np.int64).sum() + n)
    return synth.unpack_vocabulary(host), ck


def max_over_ranks(dist, device, world: int, seconds: float) -> float:
    """The timed region's wall time: max over ranks (bench contract)."""
    import torch

    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=768, help="independent streams per GPU")
    ap.add_argument("--groups", type=int, default=3,
                    help="stream groups per GPU, each on its own HIP stream (their kernels overlap)")
    ap.add_argument("--camera", default="euroc")
    ap.add_argument("--nfeatures", type=int, default=1000)
    ap.add_argument("--gf-budget", type=int, default=100)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--lba-batch", type=int, default=64, help="local-BA windows solved together (0: skip)")
    ap.add_argument("--single-stream-steps", type=int, default=20,
                    help="also time one stream alone (per-frame latency of a single sequence)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from gf_orb_slam_amd import synth
    from gf_orb_slam_amd.pipeline import FrontEnd

    cam = args.camera
    w, h = synth.CAMERAS[cam][:2]
    B = args.batch
    G = max(1, args.groups)
    if B % G:
        raise SystemExit(f"--batch {B} must be a multiple of --groups {G}")
    Bg = B // G
    # G groups of B/G streams, each a FrontEnd with its own context and HIP
    # stream: their kernels overlap, so one group's latency-bound stages (pose
    # LM, active matching) run beside another group's extraction
    fes = []
    for g in range(G):
        fe = FrontEnd(cam, args.nfeatures, Bg, 2000, gf_budget=args.gf_budget, seed=rank * G + g)
        base = rank * B + g * Bg
        frames = np.stack([synth.synth_frame(w, h, synth.frame_seed(base + b, 0)) for b in range(min(Bg, 8))])
        fe.load_frames(frames[np.arange(Bg) % len(frames)])
        fe.build_maps()
        fes.append(fe)

    # one-off exchange before timing: rank 0 broadcasts the ORB vocabulary (RCCL over xGMI)
    t_bc = time.perf_counter()
    voc_tree, voc_ck = share_startup_state(dist, "cuda", world, rank)
    torch.cuda.synchronize()
    t_bc = time.perf_counter() - t_bc
    from gf_orb_slam_amd.bow import ORBVocabulary
    vocab = ORBVocabulary(voc_tree)  # every rank holds it on its own device (D1 path)
    startup = {"vocabulary_nodes": vocab.info()["nnodes"], "broadcast_MB": round(voc_tree["desc"].nbytes * 45 / 32 / 1e6, 1),
               "broadcast_s": round(t_bc, 3), "checksum": voc_ck}

    for _ in range(args.warmup):
        for fe in fes:
            fe.step()
    for fe in fes:
        fe.sync()
        # HIP events around every launch on its group's stream, over the timed region
        fe.prof_enable(True)
        fe.prof_reset()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        for fe in fes:
            fe.step()
    for fe in fes:
        fe.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    dt = max_over_ranks(dist, "cuda", world, dt)
    prof = {}
    for fe in fes:
        for k, (ms, cnt) in fe.prof_report().items():
            a = prof.setdefault(k, [0.0, 0])
            a[0] += ms
            a[1] += cnt
        fe.prof_enable(False)
    prof_steps = args.steps
    fe = fes[0]

    frames_total = world * B * args.steps
    fps = frames_total / dt
    nk = float(np.mean([f.nkp.float().mean().item() for f in fes]))
    iters = np.concatenate([f.iters.cpu().numpy() for f in fes], axis=1).astype(np.float64)   # [2][B] LM iterations
    nedges = np.concatenate([f.nedges.cpu().numpy() for f in fes], axis=1).astype(np.float64)  # [2][B] edges
    n_active = float(np.mean([f.n_active.float().mean().item() for f in fes]))
    ninl = float(np.mean([f.ninl.float().mean().item() for f in fes]))

    # algorithmic bytes per launch for the kernels with a §8(d) formula
    kb = kernel_bytes(cam, args.nfeatures)
    per_launch_bytes = {k: kb[k] * Bg for k in ("k_resize", "k_blur_fast", "k_describe")}
    # pose LM: N_e * 40 B per LM iteration per problem, summed over the launch
    per_launch_bytes["k_pose_opt"] = float((nedges * iters).sum(axis=1).mean() * 40.0) / G
    per_kernel = {k: {"avg_ms": v[0] / max(v[1], 1), "launches": v[1], "ms_per_step": v[0] / prof_steps}
                  for k, v in prof.items()}
    # the roofline is priced on the kernel with the largest total time that has
    # an algorithmic byte count; a latency-bound stage that ranks above it
    # (one wave per frame walking a sequential loop: active matching) is named
    # beside it, since an HBM roofline says nothing about it
    top = max(prof, key=lambda k: prof[k][0])
    priced = [k for k in prof if k in per_launch_bytes]
    dom = max(priced, key=lambda k: prof[k][0]) if priced else top
    avg_s = prof[dom][0] / prof[dom][1] / 1e3
    # HBM bytes per launch from the committed rocprofv3 PMC passes of this code
    # (profiles/r01/pmc_traffic.json, scripts/pmc_extract.sh), when taken at this batch
    traffic = None
    try:
        pmc = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "r01",
                                          "pmc_traffic.json")))
        if pmc.get("batch") == Bg and dom in pmc.get("kernels", {}):
            traffic = round(pmc["kernels"][dom]["traffic_bytes"])
    except (OSError, ValueError, KeyError):
        traffic = None
    if dom in per_launch_bytes:
        achieved = per_launch_bytes[dom] / avg_s / 1e9
        roof = {"kernel": dom, "bound": "hbm", "achieved": round(achieved, 2), "peak": 8000.0, "unit": "GB/s",
                "frac": round(achieved / 8000.0, 5), "traffic": traffic,
                "traffic_source": "profiles/r01/pmc_traffic.json (FETCH_SIZE+WRITE_SIZE per launch)" if traffic else None,
                "algorithmic_bytes_per_launch": per_launch_bytes[dom], "frames_per_launch": Bg,
                "avg_launch_ms": round(avg_s * 1e3, 4)}
    else:
        roof = {"kernel": dom, "bound": "hbm", "achieved": None, "peak": 8000.0, "unit": "GB/s", "frac": None,
                "traffic": None, "avg_launch_ms": round(avg_s * 1e3, 4)}
    if top != dom:
        roof["largest_kernel"] = {"kernel": top, "avg_launch_ms": round(prof[top][0] / prof[top][1], 4),
                                  "bound": "latency: one wave per frame runs the reference's sequential "
                                           "selection loop; its time stretches while it waits for CUs "
                                           "beside the other groups' extraction"}
    ext_ms = sum(prof[k][0] for k in ("k_resize", "k_blur_fast", "k_fast_cells", "k_select", "k_describe") if k in prof)
    ext_bw = kb["extract_total"] * B * prof_steps / (ext_ms / 1e3) / 1e9 if ext_ms else None
    pose_ms = prof.get("k_pose_opt", (0.0, 1))
    pose_avg_ms = pose_ms[0] / max(pose_ms[1], 1)
    mean_iters = float(iters.mean())

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
        "data": "synthetic (seeded 752x480 frames + synthetic 2000-point local maps; no dataset reachable)",
        "config": {"workload": f"config 2: {cam} {w}x{h}, {args.nfeatures} feats, GF budget {args.gf_budget}, "
                               f"{B} streams/GPU in {G} groups; step = extract + motion model + SearchByProjection(last frame) + "
                               f"PoseOptimization + G1-G7 active map matching + PoseOptimization",
                   "streams_per_gpu": B, "stream_groups": G, "parallelism": f"{B} streams x {world} ranks"},
        "startup": startup,
        "roofline": roof,
        "pose_opt": {"ms_per_iter": round(pose_avg_ms / max(mean_iters, 1e-9), 5),
                     "ms_per_iter_per_problem": round(pose_avg_ms / max(mean_iters * Bg, 1e-9), 6),
                     "avg_launch_ms": round(pose_avg_ms, 4), "mean_iterations": round(mean_iters, 2),
                     "mean_edges": [round(float(x), 1) for x in nedges.mean(axis=1)],
                     "note": "ms_per_iter = launch time / mean LM iterations (all B problems run concurrently)"},
        "extraction_stage": {"ms_per_frame": round(ext_ms / (B * prof_steps), 5),
                             "algorithmic_GBps": round(ext_bw, 2) if ext_bw else None},
        "kernels_note": f"HIP events per launch over the timed region; each launch covers one group ({Bg} streams) "
                        f"and the {G} groups' launches overlap, so ms_per_step sums exceed the wall time per step",
        "kernels": {k: {"avg_ms": round(v["avg_ms"], 4), "launches": v["launches"],
                        "ms_per_step": round(v["ms_per_step"], 4)} for k, v in per_kernel.items()},
        "avg_keypoints": nk,
        "avg_active_matches": n_active,
        "avg_inliers": ninl,
    }
    if rank == 0 and args.single_stream_steps > 0:
        out["single_stream"] = single_stream(cam, args.nfeatures, args.gf_budget, args.single_stream_steps)
    if rank == 0 and args.lba_batch > 0:
        out["local_ba"] = lba_leg(args.lba_batch, cpu=not args.no_cpu_baseline)
    if rank == 0 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(cam, args.nfeatures)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
