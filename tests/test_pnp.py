"""Relocalisation PnP: PnPsolver (src/PnPsolver.cc) — EPnP minimal sets in
RANSAC, Refine() on the best inlier set, iterate()/bNoMore bookkeeping and the
std::rand() draws (DUtils::Random::RandomInt). OpenCV's SVD/solve/invert are
restated (oracle/pnp.cpp), so parity is unpinned against OpenCV itself; the CPU
tests pin the oracle to ground-truth poses and to the reference's control flow,
the GPU tests hold the device path to the oracle bit for bit (poses, inlier
masks, counts, flags and the caller's rand() state)."""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
from gf_orb_slam_amd._lib import check, lib, ptr
from gf_orb_slam_amd.pnp import (GF_PNP_FOUND, GF_PNP_NOMORE, GF_PNP_REFINED, PNP_STATE_DTYPE, RNG_DTYPE,
                                 pnp_params)

EUROC_K = (458.654, 457.296, 367.215, 248.375)
RELOC = dict(probability=0.99, min_inliers=10, max_iterations=300, min_set=4, epsilon=0.5, th2=5.991)  # Tracking.cc:3917


def _rot(a, b, c):
    ca, sa, cb, sb, cc, sc = np.cos(a), np.sin(a), np.cos(b), np.sin(b), np.cos(c), np.sin(c)
    Rz = np.array([[ca, -sa, 0], [sa, ca, 0], [0, 0, 1]])
    Rx = np.array([[1, 0, 0], [0, cb, -sb], [0, sb, cb]])
    Ry = np.array([[cc, 0, sc], [0, 1, 0], [-sc, 0, cc]])
    return Rz @ Rx @ Ry


def scene(n, seed, outliers=0.3, noise=0.5, K=EUROC_K):
    """n world points seen by a camera at a random pose: projections with
    Gaussian pixel noise, `outliers` of them displaced by 20-60 px, octave
    U{0..7} (sigma^2 = 1.2^(2 oct))."""
    rng = np.random.default_rng(seed)
    R = _rot(*rng.uniform(-0.4, 0.4, 3))
    t = rng.uniform(-0.5, 0.5, 3)
    Pc = np.stack([rng.uniform(-3, 3, n), rng.uniform(-2, 2, n), rng.uniform(2, 8, n)], 1)
    Pw = (Pc - t) @ R
    fx, fy, cx, cy = K
    uv = np.stack([fx * Pc[:, 0] / Pc[:, 2] + cx, fy * Pc[:, 1] / Pc[:, 2] + cy], 1) + rng.normal(0, noise, (n, 2))
    octave = rng.integers(0, 8, n)
    s2 = (1.2 ** (2 * octave)).astype(np.float32)
    bad = rng.random(n) < outliers
    uv[bad] += rng.uniform(20, 60, (bad.sum(), 2)) * rng.choice([-1, 1], (bad.sum(), 2))
    T = np.eye(4)
    T[:3, :3], T[:3, 3] = R, t
    return Pw.astype(np.float32), uv.astype(np.float32), s2, np.asarray(K, np.float32), T, bad


def _params(**kw):
    return pnp_params(**{**RELOC, **kw})


# ------------------------------------------------------------------ CPU
@pytest.mark.parametrize("n,seed", [(40, 1), (120, 2), (400, 3), (1000, 4)])
def test_oracle_recovers_pose_and_inliers(n, seed):
    P, uv, s2, K, T, bad = scene(n, seed)
    Ts, inl, ninl, fl, _ = O.pnp_run(P, uv, s2, K, _params(), 7, [300])
    assert fl[0] & GF_PNP_FOUND and fl[0] & GF_PNP_REFINED
    assert np.abs(Ts[0][:3, :3] - T[:3, :3]).max() < 2e-3 and np.abs(Ts[0][:3, 3] - T[:3, 3]).max() < 2e-2
    assert np.array_equal(inl[0].astype(bool), ~bad) and ninl[0] == (~bad).sum()


def test_oracle_too_few_correspondences():
    """N < mRansacMinInliers: bNoMore, no pose, no rand() draws (:145-149)."""
    P, uv, s2, K, _, _ = scene(9, 5)
    _, _, ninl, fl, rc = O.pnp_run(P, uv, s2, K, _params(), 3, [5, 5])
    assert list(fl) == [GF_PNP_NOMORE] * 2 and list(ninl) == [0, 0] and list(rc) == [0, 0]


def test_oracle_iteration_accounting():
    """Four draws per iteration; a call runs while mnIterations < max or the
    call's count is not reached (:154); bNoMore once max is reached."""
    P, uv, s2, K, _, _ = scene(12, 6, outliers=0.6)  # fewer good points than mRansacMinInliers
    st = np.zeros(1, PNP_STATE_DTYPE)
    check(lib().gf_pnp_init(12, ptr(_params()), ptr(st)))
    mx = int(st["max_iterations"][0])
    _, _, _, fl, rc = O.pnp_run(P, uv, s2, K, _params(), 11, [2, 3, 5])
    assert rc[0] == 4 * max(2, mx) and rc[1] - rc[0] == 4 * 3 and rc[2] - rc[1] == 4 * 5
    assert all(f == GF_PNP_NOMORE for f in fl)


@pytest.mark.parametrize("n", [0, 9, 10, 12, 20, 100, 5000])
def test_set_ransac_parameters_matches_oracle(n):
    """gf_pnp_init (library host code) == the oracle's SetRansacParameters."""
    for kw in (RELOC, dict(probability=0.99, min_inliers=8, max_iterations=300, min_set=4, epsilon=0.4, th2=5.991)):
        a = np.zeros(1, PNP_STATE_DTYPE)
        b = np.zeros(1, PNP_STATE_DTYPE)
        check(lib().gf_pnp_init(n, ptr(pnp_params(**kw)), ptr(a)))
        assert O.orc().orc_pnp_init(n, O._p(pnp_params(**kw)), O._p(b)) == 0
        assert a.tobytes() == b.tobytes()


# ------------------------------------------------------------------ GPU
def _rng_after(seed, calls):
    g = np.zeros(1, RNG_DTYPE)
    check(lib().gf_rng_seed(ptr(g), ctypes.c_uint32(seed)))
    if calls:
        sink = np.zeros(calls, np.int32)  # held: gf_rng_next writes `calls` values into it
        check(lib().gf_rng_next(ptr(g), ptr(sink), calls))
    return g


CASES = [(12, 1, 0.6, [5, 5, 5]), (40, 2, 0.3, [5, 5, 5, 5, 300]), (120, 3, 0.5, [5, 5, 5, 300]),
         (400, 4, 0.3, [300]), (1000, 5, 0.45, [5, 5]), (9, 6, 0.0, [5]), (250, 7, 0.0, [5])]


@pytest.mark.gpu
@pytest.mark.parametrize("n,seed,outl,calls", CASES)
def test_pnp_iterate_gpu_bit_exact(n, seed, outl, calls):
    from gf_orb_slam_amd.matcher import default_context

    P, uv, s2, K, _, _ = scene(n, seed, outliers=outl)
    To, io, no, fo, ro = O.pnp_run(P, uv, s2, K, _params(), 1000 + seed, calls)
    ctx = default_context()
    st = np.zeros(1, PNP_STATE_DTYPE)
    check(lib().gf_pnp_init(n, ptr(_params()), ptr(st)))
    g = _rng_after(1000 + seed, 0)
    bm = np.zeros(max(n, 1), np.uint8)
    for c, it in enumerate(calls):
        T = np.zeros(16, np.float32)
        inl = np.zeros(max(n, 1), np.uint8)
        ni = np.zeros(1, np.int32)
        fl = np.zeros(1, np.int32)
        check(lib().gf_pnp_iterate(ctx.handle, ptr(P), ptr(uv), ptr(s2), ptr(K), ptr(st), ptr(bm), it, ptr(g), ptr(T),
                                   ptr(inl), ptr(ni), ptr(fl)))
        assert fl[0] == fo[c] and ni[0] == no[c], (c, fl[0], fo[c], ni[0], no[c])
        assert T.tobytes() == To[c].reshape(16).tobytes()
        assert np.array_equal(inl[:n], io[c])
        assert g.tobytes() == _rng_after(1000 + seed, int(ro[c])).tobytes()


@pytest.mark.gpu
def test_pnp_batch_dev_matches_oracle():
    """gf_pnp_iterate_dev: 24 independent solvers (ragged sizes, own rand()
    streams) in one launch, two successive calls."""
    import torch

    from gf_orb_slam_amd.matcher import default_context

    dev = torch.device("cuda:0")
    sizes = [15, 40, 300, 9, 120, 800, 60, 33] * 3
    cap = max(sizes)
    B = len(sizes)
    p3 = np.zeros((B, cap, 3), np.float32)
    p2 = np.zeros((B, cap, 2), np.float32)
    s2 = np.ones((B, cap), np.float32)
    st = np.zeros(B, PNP_STATE_DTYPE)
    rng = np.zeros(B, RNG_DTYPE)
    ref = []
    calls = [5, 300]
    for b, n in enumerate(sizes):
        P, uv, s, K, _, _ = scene(n, 100 + b, outliers=0.4)
        p3[b, :n], p2[b, :n], s2[b, :n] = P, uv, s
        check(lib().gf_pnp_init(n, ptr(_params()), ptr(st[b:b + 1])))
        rng[b:b + 1] = _rng_after(500 + b, 0)
        ref.append(O.pnp_run(P, uv, s, K, _params(), 500 + b, calls))
    K = np.asarray(EUROC_K, np.float32)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)).to(dev)  # noqa: E731
    d3, d2, ds, dst, drng = t(p3), t(p2), t(s2), t(st), t(rng)
    dbm = torch.zeros(B * cap, dtype=torch.uint8, device=dev)
    dT = torch.zeros(B * 16, dtype=torch.float32, device=dev)
    dinl = torch.zeros(B * cap, dtype=torch.uint8, device=dev)
    dn = torch.zeros(B, dtype=torch.int32, device=dev)
    dfl = torch.zeros(B, dtype=torch.int32, device=dev)
    ctx = default_context()
    for c, it in enumerate(calls):
        check(lib().gf_pnp_iterate_dev(ctx.handle, B, ptr(d3), ptr(d2), ptr(ds), cap, ptr(K), ptr(dst), ptr(dbm), it,
                                       300, ptr(drng), ptr(dT), ptr(dinl), ptr(dn), ptr(dfl), ctx.stream))
        check(lib().gf_ctx_sync(ctx.handle))
        T = dT.cpu().numpy().reshape(B, 16)
        inl = dinl.cpu().numpy().reshape(B, cap)
        for b, n in enumerate(sizes):
            To, io, no, fo, ro = ref[b]
            assert dfl[b].item() == fo[c] and dn[b].item() == no[c], (b, c)
            assert T[b].tobytes() == To[c].reshape(16).tobytes(), (b, c)
            assert np.array_equal(inl[b, :n], io[c]), (b, c)
        g = drng.cpu().numpy().view(RNG_DTYPE)
        for b in range(B):
            assert g[b:b + 1].tobytes() == _rng_after(500 + b, int(ref[b][4][c])).tobytes(), (b, c)


@pytest.mark.gpu
def test_pnpsolver_class_keypoint_indexing():
    """The PnPsolver mirror: NULL / bad map points are skipped (ctor :50-72) and
    vbInliers comes back indexed by keypoint."""
    from gf_orb_slam_amd.orb import KEYPOINT_DTYPE
    from gf_orb_slam_amd.pnp import PnPsolver, Rand

    P, uv, s2, K, T, bad = scene(200, 9)
    nk = 260
    kps = np.zeros(nk, KEYPOINT_DTYPE)
    pos = np.full((nk, 3), np.nan, np.float32)
    slot = np.random.default_rng(0).permutation(nk)[:200]
    kps["x"][slot], kps["y"][slot] = uv[:, 0], uv[:, 1]
    octave = np.round(np.log(s2) / np.log(1.44)).astype(np.int32)
    kps["octave"][slot] = octave
    pos[slot] = P
    flag_bad = np.zeros(nk, bool)
    flag_bad[slot[:5]] = True
    level_s2 = (1.2 ** (2 * np.arange(8))).astype(np.float32)
    solver = PnPsolver(kps, pos, level_s2, K, bad=flag_bad)
    solver.set_ransac_parameters(0.99, 10, 300, 4, 0.5, 5.991)
    Tcw, no_more, vb, ninl = solver.iterate(5, Rand(3))
    assert Tcw is not None and np.abs(Tcw[:3, 3] - T[:3, 3]).max() < 2e-2
    expect = np.zeros(nk, bool)
    expect[slot[5:]] = ~bad[5:]
    assert np.array_equal(vb, expect) and ninl == expect.sum()
