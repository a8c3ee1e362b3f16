"""GPU parity of LocalBundleAdjustment (row B1) with the CPU oracle.

Tolerance (north_star, floating point): keyframe poses and map points agree to
1e-5 relative (|d| <= 1e-5 * max(1, |v|) per entry); outlier flags of both
optimize() rounds and the iteration counts are identical. Not bit-exact: the
reference's CHOLMOD solve is unpinned and the device sums the Schur product
in MFMA order (oracle/lba.cpp header)."""
import numpy as np
import pytest

import oracle_lib as O
from gf_orb_slam_amd._lib import GFError
from gf_orb_slam_amd.optimizer import LocalBAPlan, local_bundle_adjustment
from gf_orb_slam_amd.synth import synth_lba_problem

pytestmark = pytest.mark.gpu
RTOL = 1e-5


def _close(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.all(np.abs(a - b) <= RTOL * np.maximum(1.0, np.abs(b)))


def _check(g, o):
    Tg, Xg, og, ig = g
    To, Xo, oo, io = o
    assert ig == io, (ig, io)
    assert np.array_equal(og, oo), (np.nonzero(og != oo)[0][:10], og.sum(), oo.sum())
    assert _close(Tg, To), np.abs(Tg - To).max()
    assert _close(Xg, Xo), np.abs(Xg - Xo).max()


CASES = [(1, 3, 40), (2, 6, 300), (3, 10, 1000), (4, 20, 3000), (5, 32, 2000), (6, 1, 100)]


@pytest.mark.parametrize("seed,nkf,npts", CASES)
def test_local_ba_matches_oracle(seed, nkf, npts):
    p = synth_lba_problem(seed, nkf, npts)
    _check(local_bundle_adjustment(p), O.local_ba(p))


def test_local_ba_max_local_keyframes():
    """32 local keyframes (the limit, n = 192): k_ba_solve's triangle fills the
    LDS, so the trailing update reads its panel values from the triangle
    itself instead of the staged copy."""
    p = synth_lba_problem(7, 33, 1500, nfixed=0)  # keyframe 0 fixed: 32 free
    assert int((np.asarray(p["kf_kind"]) == 0).sum()) == 32
    _check(local_bundle_adjustment(p), O.local_ba(p))


def test_local_ba_batch_matches_oracle():
    probs = [synth_lba_problem(20 + i, n, m) for i, (n, m) in enumerate([(8, 500), (20, 3000), (4, 60), (12, 1500)])]
    plan = LocalBAPlan(probs)
    steps = plan.solve()
    assert 0 < steps <= 400
    for g, p in zip(plan.results(), probs):
        _check(g, O.local_ba(p))
    # a second solve starts again from the uploaded state
    plan.solve()
    for g, p in zip(plan.results(), probs):
        _check(g, O.local_ba(p))
    plan.close()


def test_local_ba_edge_cases():
    p = synth_lba_problem(3, 4, 30)
    empty = dict(p, edge_pt=p["edge_pt"][:0], edge_kf=p["edge_kf"][:0], edge_z=p["edge_z"][:0],
                 edge_inv_sigma2=p["edge_inv_sigma2"][:0])
    _check(local_bundle_adjustment(empty), O.local_ba(empty))
    fixed = dict(p, kf_kind=np.full_like(p["kf_kind"], 2))  # points only
    _check(local_bundle_adjustment(fixed), O.local_ba(fixed))
    noisy = synth_lba_problem(31, 5, 200, noise_px=0.5, outlier_frac=0.4)
    _check(local_bundle_adjustment(noisy), O.local_ba(noisy))


def test_local_ba_rejects_bad_graphs():
    p = synth_lba_problem(3, 4, 30)
    order = np.r_[1:len(p["edge_pt"]), 0]  # edges of point 0 split
    with pytest.raises(GFError):
        local_bundle_adjustment(dict(p, edge_pt=p["edge_pt"][order], edge_kf=p["edge_kf"][order],
                                     edge_z=p["edge_z"][order], edge_inv_sigma2=p["edge_inv_sigma2"][order]))
    big = synth_lba_problem(4, 34, 200, nfixed=0)  # 33 local keyframes
    with pytest.raises(GFError):
        local_bundle_adjustment(big)


@pytest.mark.parametrize("seed,nkf,npts", [(4, 20, 3000), (2, 6, 300)])
def test_local_ba_force_stop(seed, nkf, npts):
    """setForceStopFlag (Optimizer.cc:1579-1580): g2o checks terminate()
    before every iteration (sparse_optimizer.cpp:376), so a flag raised
    before the solve runs no iteration of optimize(5) nor of optimize(10);
    poses and points stay as given and only the depth test can flag an edge
    (the edges' errors were never computed; taken as 0). The result equals the
    oracle capped at (0, 0) iterations."""
    import ctypes

    p = synth_lba_problem(seed, nkf, npts)
    g = local_bundle_adjustment(p, stop_flag=ctypes.c_uint8(1))
    assert list(g[3]) == [0, 0], g[3]
    _check(g, O.local_ba(p, its=(0, 0)))
    free = local_bundle_adjustment(p, stop_flag=ctypes.c_uint8(0))
    _check(free, O.local_ba(p))
