"""GPU parity of the pose LM (rows P1-P4) with the CPU oracle.

Tolerance (north_star, floating point): poses agree to 1e-5 relative
(|dT| <= 1e-5 * max(1, |T|) per entry); outlier flags, inlier counts and LM
iteration counts are identical. The device keeps the oracle's summation order
(edge-ordered accumulators), so most problems also come out bit-identical;
the only expected ulp sources are libm sin/cos/pow inside the exp map.
"""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
from gf_orb_slam_amd._lib import check, lib, ptr
from gf_orb_slam_amd.matcher import MAP_POINT_DTYPE, Frame, FrameInfo
from gf_orb_slam_amd.optimizer import POSE_EDGE_DTYPE, Optimizer, inv_level_sigma2
from gf_orb_slam_amd.orb import KEYPOINT_DTYPE, default_context
from gf_orb_slam_amd.synth import synth_pose_problem

pytestmark = pytest.mark.gpu
POSE_RTOL = 1e-5


def _oracle(T0, edges, cam):
    _, _, fx, fy, cx, cy = cam
    n = len(edges)
    if n == 0:
        return O.pose_opt(T0, np.zeros((0, 3)), np.zeros((0, 2)), np.zeros(0, np.int32), np.ones(1, np.float32), fx,
                          fy, cx, cy)
    return O.pose_opt(T0, edges["X"], edges["z"], np.arange(n, dtype=np.int32), edges["inv_sigma2"], fx, fy, cx, cy)


def _assert_pose(Tg, To):
    tol = POSE_RTOL * np.maximum(1.0, np.abs(To))
    assert np.all(np.abs(Tg.astype(np.float64) - To) <= tol), np.abs(Tg - To).max()


CASES = [(s, n) for s, n in [(1, 0), (2, 1), (3, 5), (4, 9), (5, 10), (6, 63), (7, 64), (8, 65), (9, 128), (10, 200),
                             (11, 400), (12, 1000), (13, 2500)]]


@pytest.mark.parametrize("seed,n", CASES)
def test_pose_opt_matches_oracle(seed, n):
    _, T0, edges, cam = synth_pose_problem(seed, max(n, 1), noise_px=1.0, outlier_frac=0.1)
    edges = edges[:n]
    _, _, fx, fy, cx, cy = cam
    Tg, og, ng, ig = Optimizer.pose_opt_edges(T0, edges, fx, fy, cx, cy)
    To, oo, no, io = _oracle(T0, edges, cam)
    assert ng == no and ig == io
    assert np.array_equal(og, oo)
    _assert_pose(Tg, To)


def test_pose_opt_bit_exact_fraction():
    """Report (and bound) how often the device result is bit-identical."""
    exact = 0
    for seed in range(100, 140):
        _, T0, edges, cam = synth_pose_problem(seed, 300, noise_px=1.0, outlier_frac=0.1)
        _, _, fx, fy, cx, cy = cam
        Tg, og, ng, ig = Optimizer.pose_opt_edges(T0, edges, fx, fy, cx, cy)
        To, oo, no, io = _oracle(T0, edges, cam)
        assert ng == no and ig == io and np.array_equal(og, oo)
        _assert_pose(Tg, To)
        exact += int(np.array_equal(Tg, To))
    print(f"bit-identical poses: {exact}/40")
    assert exact >= 20


def test_pose_opt_large_outlier_ratio_and_far_init():
    _, T0, edges, cam = synth_pose_problem(77, 500, noise_px=2.0, outlier_frac=0.4, rot_deg=3.0, trans=0.05)
    _, _, fx, fy, cx, cy = cam
    Tg, og, ng, ig = Optimizer.pose_opt_edges(T0, edges, fx, fy, cx, cy)
    To, oo, no, io = _oracle(T0, edges, cam)
    assert ng == no and ig == io and np.array_equal(og, oo)
    _assert_pose(Tg, To)


def test_pose_opt_batch_dev_matches_oracle():
    import torch

    sizes = [0, 7, 64, 150, 333, 800, 1200, 65, 10, 2048]
    stride = 2048
    probs = [synth_pose_problem(500 + i, max(n, 1)) for i, n in enumerate(sizes)]
    E = np.zeros((len(sizes), stride), POSE_EDGE_DTYPE)
    T = np.zeros((len(sizes), 4, 4), np.float32)
    for i, (n, (_, T0, edges, cam)) in enumerate(zip(sizes, probs)):
        E[i, :n] = edges[:n]
        T[i] = T0
    cam = probs[0][3]
    _, _, fx, fy, cx, cy = cam
    dev = torch.device("cuda:0")
    dE = torch.from_numpy(E.view(np.uint8).reshape(-1)).to(dev)
    dT = torch.from_numpy(T).to(dev)
    dN = torch.tensor(sizes, dtype=torch.int32, device=dev)
    dO = torch.zeros(len(sizes) * stride, dtype=torch.uint8, device=dev)
    dI = torch.zeros(len(sizes), dtype=torch.int32, device=dev)
    dIt = torch.zeros(len(sizes), dtype=torch.int32, device=dev)
    ctx = default_context()
    Optimizer.pose_opt_batch_dev(dT, dE, dN, stride, fx, fy, cx, cy, dO, dI, dIt, ctx=ctx)
    check(lib().gf_ctx_sync(ctx.handle))
    Tg, og, ng, ig = dT.cpu().numpy(), dO.cpu().numpy().reshape(len(sizes), stride), dI.cpu().numpy(), dIt.cpu().numpy()
    for i, (n, (_, T0, edges, _c)) in enumerate(zip(sizes, probs)):
        To, oo, no, io = _oracle(T0, edges[:n], cam)
        assert ng[i] == no and ig[i] == io, i
        assert np.array_equal(og[i, :n], oo), i
        _assert_pose(Tg[i], To)


def _frame_problem(seed, nkp, nmatch, cam_name="euroc"):
    """Keypoints + kp2mp + per-frame map for the frames_dev path."""
    _, T0, edges, cam = synth_pose_problem(seed, nmatch, camera=cam_name)
    rng = np.random.default_rng(seed + 1)
    kp_idx = np.sort(rng.choice(nkp, nmatch, replace=False))
    mp_ids = rng.permutation(nmatch)  # map order differs from keypoint order
    invs = inv_level_sigma2()
    kps = np.zeros(nkp, KEYPOINT_DTYPE)
    kps["x"] = rng.uniform(0, cam[0], nkp)
    kps["y"] = rng.uniform(0, cam[1], nkp)
    kps["octave"] = rng.integers(0, 8, nkp)
    kp2mp = np.full(nkp, -1, np.int32)
    mp = np.zeros(nmatch, MAP_POINT_DTYPE)
    for j, (k, m) in enumerate(zip(kp_idx, mp_ids)):
        kps["x"][k], kps["y"][k] = edges["z"][j]
        kp2mp[k] = m
        mp["pos"][m] = edges["X"][j]
    ordered = np.zeros(nmatch, POSE_EDGE_DTYPE)
    ordered["X"] = mp["pos"][kp2mp[kp_idx]]
    ordered["z"] = np.c_[kps["x"][kp_idx], kps["y"][kp_idx]]
    ordered["inv_sigma2"] = invs[kps["octave"][kp_idx]]
    return T0, kps, kp2mp, mp, ordered, kp_idx, cam


def test_pose_opt_frames_dev_matches_oracle():
    import torch

    specs = [(900, 1000, 300), (901, 1000, 40), (902, 2000, 1200), (903, 1000, 5)]
    kp_stride, map_stride = 2048, 1500
    dev = torch.device("cuda:0")
    F = len(specs)
    K = np.zeros((F, kp_stride), KEYPOINT_DTYPE)
    NK = np.zeros(F, np.int32)
    KM = np.full((F, kp_stride), -1, np.int32)
    M = np.zeros((F, map_stride), MAP_POINT_DTYPE)
    T = np.zeros((F, 4, 4), np.float32)
    probs = []
    for f, (seed, nkp, nm) in enumerate(specs):
        T0, kps, kp2mp, mp, ordered, kp_idx, cam = _frame_problem(seed, nkp, nm)
        K[f, :nkp], NK[f], KM[f, :nkp], M[f, :nm], T[f] = kps, nkp, kp2mp, mp, T0
        probs.append((T0, ordered, kp_idx, cam))
    out0 = np.full((F, kp_stride), 7, np.uint8)  # sentinel: unmatched keypoints must stay untouched
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev)
    dK, dKM, dM, dO = t(K), t(KM), t(M), t(out0)
    dNK = torch.from_numpy(NK).to(dev)
    dT = torch.from_numpy(T).to(dev)
    dI = torch.zeros(F, dtype=torch.int32, device=dev)
    invs = inv_level_sigma2()
    cam = probs[0][3]
    _, _, fx, fy, cx, cy = cam
    ctx = default_context()
    check(lib().gf_pose_opt_frames_dev(ctx.handle, F, ptr(dT), ptr(dK), ptr(dNK), kp_stride, ptr(dKM), ptr(dM),
                                       map_stride, ptr(invs), len(invs), ctypes.c_float(fx), ctypes.c_float(fy),
                                       ctypes.c_float(cx), ctypes.c_float(cy), ptr(dO), ptr(dI), None, None,
                                       ctx.stream))
    check(lib().gf_ctx_sync(ctx.handle))
    Tg, og, ng = dT.cpu().numpy(), dO.cpu().numpy().reshape(F, kp_stride), dI.cpu().numpy()
    for f, (T0, ordered, kp_idx, _c) in enumerate(probs):
        To, oo, no, _ = _oracle(T0, ordered, cam)
        assert ng[f] == no
        assert np.array_equal(og[f, kp_idx], oo)
        mask = np.ones(kp_stride, bool)
        mask[kp_idx] = False
        assert np.all(og[f, mask] == 7)
        _assert_pose(Tg[f], To)


def test_frame_mirror_PoseOptimization():
    T0, kps, kp2mp, mp, ordered, kp_idx, cam = _frame_problem(950, 1000, 250)
    w, h, fx, fy, cx, cy = cam
    F = Frame(kps, np.zeros((len(kps), 32), np.uint8), FrameInfo.make(w, h, fx, fy, cx, cy), Tcw=T0)
    F.mvpMapPoints[:] = kp2mp
    nin = Optimizer.PoseOptimization(F, map_pos=mp["pos"])
    To, oo, no, _ = _oracle(T0, ordered, cam)
    assert nin == no
    assert np.array_equal(F.mvbOutlier[kp_idx], oo)
    _assert_pose(F.mTcw, To)
