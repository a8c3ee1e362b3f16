"""Monocular initialisation: Initializer::Initialize (src/Initializer.cc:44-132)
— the 8-point sets from std::rand(), the H and F RANSAC searches, the
H-vs-F ratio and ReconstructH / ReconstructF with CheckRT. OpenCV's float SVD,
3x3 inverse / determinant and MatExpr scalings are restated (oracle/
initializer.cpp, docs/ORACLE_ASSUMPTIONS.md A16/A17): parity is unpinned
against OpenCV itself. The CPU tests pin the oracle to ground-truth two-view
geometry and to the reference's control flow (rand() accounting, the < 8
matches guard, the failure on a pure rotation); the GPU tests hold the device
path to the oracle bit for bit (every result field, vP3D, vbTriangulated and
the caller's rand() state)."""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
from gf_orb_slam_amd._lib import GFError, check, lib, ptr
from gf_orb_slam_amd.pnp import RNG_DTYPE
from gf_orb_slam_amd.synth import synth_two_view


def _rng(seed):
    r = np.zeros(1, RNG_DTYPE)
    check(lib().gf_rng_seed(ptr(r), ctypes.c_uint32(seed)))
    return r


def _rng_after(seed, ndraws):
    r = _rng(seed)
    if ndraws:
        out = np.zeros(ndraws, np.int32)
        check(lib().gf_rng_next(ptr(r), ptr(out), ndraws))
    return r


def _rot_err_deg(R, Rg):
    return np.degrees(np.arccos(np.clip((np.trace(np.asarray(R, np.float64).T @ Rg) - 1) / 2, -1, 1)))


# ------------------------------------------------------------------ CPU
@pytest.mark.parametrize("seed", [0, 1, 3])
def test_oracle_recovers_general_motion(seed):
    """A non-planar scene: F is kept (RH <= 0.40), R21/t21 match the ground
    truth and vP3D is the scene at |t21| = 1."""
    d = synth_two_view(seed)
    rc, res, p3d, tri = O.initialize(d["K"], d["kps1"], d["kps2"], d["matches12"], _rng(42))
    r = res[0]
    assert rc == 0 and r["model"] == 1 and r["ok"] == 1, r
    assert _rot_err_deg(r["R21"].reshape(3, 3), d["R21"]) < 1.0
    tg = d["t21"] / np.linalg.norm(d["t21"])
    assert float(r["t21"] @ tg) > 0.99
    tb = tri.astype(bool)
    assert tb.sum() >= 200
    inl = np.isfinite(d["X"][:, 0])
    assert (tb & ~inl).sum() <= 0.05 * tb.sum()  # an outlier match can fall on its epipolar line
    tb &= inl
    # the scene at |t21| = 1, up to the scale error of a minimal-set model at ~4 deg parallax
    Xs = d["X"][tb] / np.linalg.norm(d["t21"])
    scale = np.median(np.linalg.norm(p3d[tb], axis=1) / np.linalg.norm(Xs, axis=1))
    assert 0.6 < scale < 1.4
    rel = np.linalg.norm(p3d[tb] - scale * Xs, axis=1) / np.linalg.norm(p3d[tb], axis=1)
    assert np.median(rel) < 0.1


@pytest.mark.parametrize("seed", [1, 5])
def test_oracle_recovers_planar_motion(seed):
    """A planar scene: H is kept (RH > 0.40) and one of the 8 Faugeras
    hypotheses wins clearly."""
    d = synth_two_view(seed, planar=True)
    rc, res, p3d, tri = O.initialize(d["K"], d["kps1"], d["kps2"], d["matches12"], _rng(42))
    r = res[0]
    assert rc == 0 and r["model"] == 0 and r["RH"] > 0.40 and r["ok"] == 1, r
    assert _rot_err_deg(r["R21"].reshape(3, 3), d["R21"]) < 1.0
    assert float(r["t21"] @ (d["t21"] / np.linalg.norm(d["t21"]))) > 0.99
    ng = np.sort(r["ngood"])[::-1]
    assert ng[1] < 0.75 * ng[0]


def test_oracle_pure_rotation_fails():
    """No baseline: no parallax, Initialize() returns false (minParallax 1 deg)."""
    d = synth_two_view(2, baseline=0.0, rot_deg=4.0)
    rc, res, p3d, tri = O.initialize(d["K"], d["kps1"], d["kps2"], d["matches12"], _rng(42))
    assert rc == 0 and res[0]["ok"] == 0
    assert not tri.any() and not p3d.any()


def test_oracle_rand_accounting():
    """8 RandomInt draws per iteration (:80-95), nothing else."""
    d = synth_two_view(0, n_match=100, n_extra=30)
    for iters in (1, 50, 200):
        r = _rng(7)
        O.initialize(d["K"], d["kps1"], d["kps2"], d["matches12"], r, iterations=iters)
        assert r.tobytes() == _rng_after(7, 8 * iters).tobytes()


def test_oracle_too_few_matches():
    d = synth_two_view(0, n_match=7, n_extra=10, outlier_frac=0.0)
    r = _rng(3)
    rc, res, _, _ = O.initialize(d["K"], d["kps1"], d["kps2"], d["matches12"], r)
    assert rc == -1 and res[0]["nmatches"] == 7 and res[0]["model"] == -1
    assert r.tobytes() == _rng(3).tobytes()


def test_oracle_distinct_minimal_sets():
    """The sets never repeat a match within an iteration (the swap-remove of
    vAvailableIndices): with exactly 8 matches every set is a permutation of
    all of them, so every F hypothesis is the 8-point fit of all matches."""
    d = synth_two_view(4, n_match=8, n_extra=20, outlier_frac=0.0)
    rc, res, _, _ = O.initialize(d["K"], d["kps1"], d["kps2"], d["matches12"], _rng(9), iterations=20)
    r = res[0]
    assert rc == 0 and r["nmatches"] == 8 and r["ninliers_F"] >= 6 and r["iter_F"] >= 0  # rank-2 projection moves F


# ------------------------------------------------------------------ GPU
CASES = [
    dict(seed=0),
    dict(seed=1),
    dict(seed=2),  # F kept, reconstruction rejected
    dict(seed=0, planar=True),  # H, two close hypotheses: rejected
    dict(seed=1, planar=True),
    dict(seed=5, planar=True),
    dict(seed=2, baseline=0.0, rot_deg=4.0),
    dict(seed=6, outlier_frac=0.45),
    dict(seed=7, n_match=12, n_extra=4, outlier_frac=0.0),
    dict(seed=8, n_match=8, n_extra=3, outlier_frac=0.0),
    dict(seed=9, n_match=2500, n_extra=1500, noise_px=1.0),
    dict(seed=10, rot_deg=20.0, baseline=1.0),
]


def _run_gpu(d, rng_seed, iterations=200, sigma=1.0):
    from gf_orb_slam_amd.initializer import INIT_RESULT_DTYPE
    from gf_orb_slam_amd.matcher import default_context

    ctx = default_context()
    n1 = len(d["kps1"])
    r = _rng(rng_seed)
    res = np.zeros(1, INIT_RESULT_DTYPE)
    p3d = np.zeros((n1, 3), np.float32)
    tri = np.zeros(n1, np.uint8)
    K = np.ascontiguousarray(d["K"].reshape(9))
    check(lib().gf_initialize(ctx.handle, ptr(K), sigma, iterations, 50, ptr(d["kps1"]), n1, ptr(d["kps2"]),
                              len(d["kps2"]), ptr(d["matches12"]), ptr(r), ptr(res), ptr(p3d), ptr(tri)))
    return r, res, p3d, tri


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=[str(c) for c in CASES])
def test_initialize_gpu_bit_exact(case):
    d = synth_two_view(**case)
    ro = _rng(1234)
    rc, reso, p3do, trio = O.initialize(d["K"], d["kps1"], d["kps2"], d["matches12"], ro)
    assert rc == 0
    rg, resg, p3dg, trig = _run_gpu(d, 1234)
    for f in reso.dtype.names:
        assert np.array_equal(np.asarray(reso[f]).view(np.uint8), np.asarray(resg[f]).view(np.uint8)), \
            (f, reso[f], resg[f])
    assert np.array_equal(p3do.view(np.uint32), p3dg.view(np.uint32))
    assert np.array_equal(trio, trig)
    assert ro.tobytes() == rg.tobytes()


@pytest.mark.gpu
def test_initialize_gpu_iterations_and_sigma():
    d = synth_two_view(3, n_match=400)
    for iters, sigma in ((1, 1.0), (37, 1.0), (200, 2.0)):
        ro = _rng(5)
        _, reso, p3do, trio = O.initialize(d["K"], d["kps1"], d["kps2"], d["matches12"], ro, sigma=sigma,
                                           iterations=iters)
        rg, resg, p3dg, trig = _run_gpu(d, 5, iterations=iters, sigma=sigma)
        assert reso.tobytes() == resg.tobytes() and p3do.tobytes() == p3dg.tobytes()
        assert trio.tobytes() == trig.tobytes() and ro.tobytes() == rg.tobytes()


@pytest.mark.gpu
def test_initialize_gpu_argument_errors():
    d = synth_two_view(0, n_match=7, n_extra=10, outlier_frac=0.0)
    with pytest.raises(GFError):
        _run_gpu(d, 1)
    d = synth_two_view(0, n_match=50, n_extra=10)
    d["matches12"][np.nonzero(d["matches12"] >= 0)[0][0]] = len(d["kps2"])
    with pytest.raises(GFError):
        _run_gpu(d, 1)


@pytest.mark.gpu
def test_initialize_dev_matches_host_and_reports_few_matches():
    import torch

    from gf_orb_slam_amd.initializer import INIT_RESULT_DTYPE, initialize_device
    from gf_orb_slam_amd.matcher import default_context

    ctx = default_context()
    dev = torch.device("cuda:0")
    for case in (dict(seed=1), dict(seed=0, n_match=6, n_extra=9, outlier_frac=0.0)):
        d = synth_two_view(**case)
        k1 = torch.from_numpy(d["kps1"].view(np.uint8).reshape(-1, 28).copy()).to(dev)
        k2 = torch.from_numpy(d["kps2"].view(np.uint8).reshape(-1, 28).copy()).to(dev)
        m = torch.from_numpy(d["matches12"].copy()).to(dev)
        rs = torch.from_numpy(_rng(77).view(np.uint8).copy()).to(dev)
        res, p3d, tri = initialize_device(ctx, d["K"], k1, k2, m, rs)
        torch.cuda.synchronize()
        r = res.cpu().numpy().view(INIT_RESULT_DTYPE)
        ro = _rng(77)
        rc, reso, p3do, trio = O.initialize(d["K"], d["kps1"], d["kps2"], d["matches12"], ro)
        if rc == 0:
            assert r.tobytes() == reso.tobytes() and p3d.cpu().numpy().tobytes() == p3do.tobytes()
            assert tri.cpu().numpy().tobytes() == trio.tobytes()
            assert rs.cpu().numpy().tobytes() == ro.view(np.uint8).tobytes()
        else:  # fewer than 8 matches: reported, rng untouched
            assert r[0]["model"] == -1 and r[0]["nmatches"] == reso[0]["nmatches"] and r[0]["ok"] == 0
            assert rs.cpu().numpy().tobytes() == _rng(77).view(np.uint8).tobytes()


@pytest.mark.gpu
def test_initializer_class_recovers_motion():
    from gf_orb_slam_amd.initializer import Initializer
    from gf_orb_slam_amd.pnp import Rand

    d = synth_two_view(1)
    ini = Initializer(d["kps1"], d["K"], sigma=1.0, iterations=200)
    ok, R21, t21, p3d, tri = ini.initialize(d["kps2"], d["matches12"], Rand(42))
    assert ok and _rot_err_deg(R21, d["R21"]) < 1.0 and tri.sum() >= 200
    assert float(t21[:, 0] @ (d["t21"] / np.linalg.norm(d["t21"]))) > 0.99


@pytest.mark.gpu
def test_initialize_batch_dev_matches_oracle():
    """gf_initialize_batch_dev: 20 ragged problems (general, planar, pure
    rotation, outliers, fewer than 8 matches) with their own rand() streams in
    one launch set, each equal to the oracle run alone."""
    import torch

    from gf_orb_slam_amd.initializer import INIT_RESULT_DTYPE, initialize_batch_device
    from gf_orb_slam_amd.matcher import default_context

    cases = [dict(seed=s) for s in range(6)] + [dict(seed=s, planar=True) for s in range(4)] + \
        [dict(seed=3, baseline=0.0), dict(seed=4, outlier_frac=0.4), dict(seed=5, n_match=5, n_extra=9),
         dict(seed=6, n_match=30, n_extra=2), dict(seed=7, n_match=900, n_extra=100)] + \
        [dict(seed=20 + s, n_match=150 + 50 * s, n_extra=20 * s) for s in range(5)]
    ds = [synth_two_view(**c) for c in cases]
    P = len(ds)
    cap1 = max(len(d["kps1"]) for d in ds)
    cap2 = max(len(d["kps2"]) for d in ds)
    k1 = np.zeros((P, cap1, 28), np.uint8)
    k2 = np.zeros((P, cap2, 28), np.uint8)
    m = np.full((P, cap1), -1, np.int32)
    n1 = np.array([len(d["kps1"]) for d in ds], np.int32)
    n2 = np.array([len(d["kps2"]) for d in ds], np.int32)
    rs = np.stack([_rng(100 + i).view(np.uint8) for i in range(P)]).reshape(P, -1)
    for i, d in enumerate(ds):
        k1[i, :n1[i]] = d["kps1"].view(np.uint8).reshape(-1, 28)
        k2[i, :n2[i]] = d["kps2"].view(np.uint8).reshape(-1, 28)
        m[i, :n1[i]] = d["matches12"]
    dev = torch.device("cuda:0")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    rs_d = t(rs)
    res, p3d, tri = initialize_batch_device(default_context(), ds[0]["K"], t(k1), t(n1), t(k2), t(n2), t(m), rs_d)
    torch.cuda.synchronize()
    res = res.cpu().numpy().view(INIT_RESULT_DTYPE).reshape(P)
    p3d, tri, rs_d = p3d.cpu().numpy(), tri.cpu().numpy(), rs_d.cpu().numpy()
    for i, d in enumerate(ds):
        ro = _rng(100 + i)
        rc, reso, p3do, trio = O.initialize(d["K"], d["kps1"], d["kps2"], d["matches12"], ro)
        if rc != 0:  # fewer than 8 matches: reported, rng untouched
            assert res[i]["model"] == -1 and res[i]["nmatches"] == reso[0]["nmatches"], i
            assert rs_d[i].tobytes() == _rng(100 + i).tobytes(), i
            continue
        assert res[i].tobytes() == reso[0].tobytes(), (i, cases[i])
        assert p3d[i, :n1[i]].tobytes() == p3do.tobytes() and tri[i, :n1[i]].tobytes() == trio.tobytes(), i
        assert rs_d[i].tobytes() == ro.tobytes(), i
