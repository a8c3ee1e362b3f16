"""CPU oracle of the pose LM (rows P1-P4): self-consistency and recovery
properties. Parity is unpinned against the reference (no PoseOptimization
test or fixture exists upstream); these checks pin the oracle to
the algorithm's known behaviour instead."""
import numpy as np
import pytest

import oracle_lib as O
from gf_orb_slam_amd.synth import synth_pose_problem


def _solve(T, edges, cam):
    _, _, fx, fy, cx, cy = cam
    octave = np.zeros(len(edges), np.int32)
    # pass per-edge inv_sigma2 through a one-level table per edge
    return O.pose_opt(T, edges["X"], edges["z"], np.arange(len(edges), dtype=np.int32), edges["inv_sigma2"],
                      fx, fy, cx, cy) if len(edges) else O.pose_opt(T, np.zeros((0, 3)), np.zeros((0, 2)), octave,
                                                                    np.ones(1, np.float32), fx, fy, cx, cy)


def test_ldlt_matches_numpy():
    rng = np.random.default_rng(3)
    for _ in range(50):
        A = rng.standard_normal((6, 6))
        H = A @ A.T + 0.1 * np.eye(6)
        b = rng.standard_normal(6)
        ok, x = O.ldlt_solve(H, b)
        assert ok
        np.testing.assert_allclose(x, np.linalg.solve(H, b), rtol=1e-9, atol=1e-10)


def test_ldlt_rejects_indefinite():
    H = np.diag([1.0, -2.0, 3.0, 4.0, 5.0, 6.0])
    ok, _ = O.ldlt_solve(H, np.ones(6))
    assert not ok


def test_ldlt_reads_lower_triangle_only():
    rng = np.random.default_rng(4)
    A = rng.standard_normal((6, 6))
    H = A @ A.T + np.eye(6)
    Hu = np.tril(H) + np.triu(rng.standard_normal((6, 6)), 1)  # garbage above the diagonal
    assert np.array_equal(O.ldlt_solve(H, np.ones(6))[1], O.ldlt_solve(Hu, np.ones(6))[1])


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_noise_free_recovers_pose(seed):
    T_true, T0, edges, cam = synth_pose_problem(seed, 200, noise_px=0.0, outlier_frac=0.0)
    T, outl, ninl, iters = _solve(T0, edges, cam)
    assert ninl == 200 and outl.sum() == 0
    np.testing.assert_allclose(T, T_true, atol=2e-5)
    assert 1 <= iters <= 32


@pytest.mark.parametrize("seed", [5, 6])
def test_outliers_flagged(seed):
    T_true, T0, edges, cam = synth_pose_problem(seed, 400, noise_px=0.5, outlier_frac=0.1)
    T, outl, ninl, _ = _solve(T0, edges, cam)
    assert ninl == 400 - outl.sum()
    assert outl.sum() >= 10  # 40 displaced 3-6 px; high octaves (small inv_sigma2) stay inliers
    assert np.abs(T[:3, 3] - T_true[:3, 3]).max() < 5e-3


def test_few_edges_single_round_and_empty():
    T_true, T0, edges, cam = synth_pose_problem(9, 8, noise_px=0.0, outlier_frac=0.0)
    T, outl, ninl, iters = _solve(T0, edges, cam)
    assert ninl == 8 and iters <= 10  # edges < 10: break after the first round
    T, outl, ninl, iters = _solve(T0, edges[:0], cam)
    assert ninl == 0 and iters == 0
    np.testing.assert_allclose(T, T0, atol=1e-6)  # quaternion round trip only
