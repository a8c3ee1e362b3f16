"""Oracle checks for the good-feature rows (G1-G7) against the reference's
own known-answer tests (tests/golden/kat_observability.json, transcribed
from test/test_Kine_1.cpp, test_Kine_2.cpp, test_Jacobian.cpp) and the
test_Greedy.cpp lazier-vs-baseline property, seeded."""
import ctypes
import json
import math
import os

import numpy as np
import pytest

import oracle_lib as O
from gf_orb_slam_amd.observability import ObsCamera

KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "kat_observability.json")))


def infnorm(A):
    return np.abs(np.asarray(A)).sum(1).max()


@pytest.mark.parametrize("case", ["kine1", "kine2"])
def test_kinematics_kat(case):
    c = KAT[case]
    ks = O.obs_predict(c["Xv"], c["dt"], c["nseg"])
    tol = KAT["tol"]
    for i, k in enumerate(ks):
        assert infnorm(np.array(k.F_Q[:]).reshape(4, 4) - c["F_Q"][i]) < tol["F_Q"]
        assert infnorm(np.array(k.F_Omg[:]).reshape(4, 3) - c["F_Omg"][i]) < tol["F_Omg"]
        assert infnorm(np.array(k.F_Q_inSeg[:]).reshape(4, 4) - c["F_Q_inSeg"][i]) < tol["F_Q_inSeg"]
        assert infnorm(np.array(k.F_Omg_inSeg[:]).reshape(4, 3) - c["F_Omg_inSeg"][i]) < tol["F_Omg_inSeg"]


def _project(Tcw, P, fu, fv, cx, cy):
    T = np.array(Tcw, np.float32).reshape(4, 4)
    Pc = (T[:3, :3] @ np.float32(P) + T[:3, 3]).astype(np.float32)
    return np.float32(fu) * Pc[0] / Pc[2] + np.float32(cx), np.float32(fv) * Pc[1] / Pc[2] + np.float32(cy)


def test_kine2_projection_kat():
    c = KAT["kine2"]
    ks = O.obs_predict(c["Xv"], c["dt"], 3)
    cam = c["camera"]
    for P, px in zip(c["landmarks"], c["pixels"]):
        u, v = _project(ks[0].Tcw[:], P, cam["f"] / cam["dx"], cam["f"] / cam["dy"], cam["cx"], cam["cy"])
        assert abs(u - px[0]) < KAT["tol"]["pixel"] and abs(v - px[1]) < KAT["tol"]["pixel"]


def test_jacobian_kat():
    c = KAT["jacobian"]
    cc = c["camera"]
    cam = ObsCamera.from_focal(cc["f"], cc["nrows"], cc["ncols"], cc["cx"], cc["cy"], cc["dx"], cc["dy"])
    ks = O.obs_predict(c["Xv"], c["dt"], 1)
    xv = np.array(ks[0].Xv[:])
    H, info, uv, valid = O.obs_build_info(cam, xv, c["landmarks"], None, False)
    for j in range(5):
        h = H[j].reshape(2, 7)
        assert infnorm(h[:, :3] - c["H13"][j]) < KAT["tol"]["H"], (j, h[:, :3])
        assert infnorm(h[:, 3:] - c["H47"][j]) < KAT["tol"]["H"], (j, h[:, 3:])
        assert abs(uv[j, 0] - c["pixels"][j][0]) < 10 and abs(uv[j, 1] - c["pixels"][j][1]) < 10
        # info block = H^T H (map path, Sigma = I)
        np.testing.assert_allclose(info[j].reshape(7, 7), h.T @ h, rtol=1e-12, atol=1e-9)


def test_logdet_matches_numpy():
    rng = np.random.default_rng(0)
    A = rng.normal(size=(50, 7, 7))
    M = A @ A.transpose(0, 2, 1) + 1e-3 * np.eye(7)
    ld = O.logdet(M)
    np.testing.assert_allclose(ld, np.linalg.slogdet(M)[1], rtol=1e-10, atol=1e-10)
    # non-PD falls back to LU log|det|
    B = rng.normal(size=(10, 7, 7))
    np.testing.assert_allclose(O.logdet(B), np.linalg.slogdet(B)[1], rtol=1e-9, atol=1e-9)


def test_rand_is_glibc():
    """orc::Rand (random_r TYPE_3) reproduces glibc's srand(1)/rand()."""
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(1)
    ref = [libc.rand() for _ in range(1000)]
    assert list(O.rand_sequence(1, 1000)) == ref


# ----------------------------------------------------------------- test_Greedy
def greedy_world(n=320, seed=1):
    """test_Greedy.cpp:81-194 fixture: 320 landmarks in a 752x480 EuRoC-like
    camera, drawn with glibc rand() from seed 1."""
    c = KAT["jacobian"]
    f, dx = 5.1369248, 0.01123325985
    cam = ObsCamera.from_focal(f, 480, 752, 367.215, 248.375, dx, dx)
    ks = O.obs_predict(c["Xv"], 0.1, 1)
    T = np.array(ks[0].Tcw[:], np.float32).reshape(4, 4)
    r = iter(O.rand_sequence(seed, 20000))
    RM = np.float32(2147483647)
    pos, oct_, score = [], [], []
    while len(pos) < n:
        P = np.array([np.float32(next(r)) / RM * 8 - 4, np.float32(next(r)) / RM * 8 - 4,
                      np.float32(next(r)) / RM * 8], np.float32)
        Pc = (T[:3, :3] @ P + T[:3, 3]).astype(np.float32)
        if Pc[2] < 0:
            continue
        u = np.float32(cam.fu) * Pc[0] / Pc[2] + np.float32(cam.cx)
        v = np.float32(cam.fv) * Pc[1] / Pc[2] + np.float32(cam.cy)
        if u < 0 or u > 752 or v < 0 or v > 480:
            continue
        oct_.append(int(np.round(np.float32(next(r)) / RM * 7)))
        next(r), next(r)  # keypoint jitter (unused by the information blocks)
        score.append(float(np.round(np.float32(next(r)) / RM * 100)))
        pos.append(P)
    sf = [np.float32(1.0)]
    for _ in range(7):
        sf.append(np.float32(sf[-1] * np.float32(1.2)))
    sigma2 = np.array([np.float32(sf[o] * sf[o]) for o in oct_], np.float32)
    H, info, uv, valid = O.obs_build_info(cam, np.array(ks[0].Xv[:]), np.array(pos), sigma2, False)
    return info, np.array(score)


def test_greedy_lazier_vs_baseline_property():
    info, score = greedy_world()
    n = len(score)
    for k in range(60, 141, 20):
        base = set(O.maxvol_select(info, score, k, 0, 1, 0).tolist())
        assert len(base) == k
        scale = float(int(np.float32(n) / np.float32(k) * math.log(1.0 / 0.1)))
        for rep in range(12):
            lazy = O.maxvol_select(info, score, k, scale, 3, 1000 + rep)
            assert len(lazy) == k
            assert len(base - set(lazy.tolist())) <= math.ceil(0.2 * k)


def test_deletion_branch():
    info, score = greedy_world()
    n = len(score)
    k = 250  # 2k > n -> maxVolDeletion_LazierGreedy
    scale = float(int(np.float32(n) / np.float32(k) * math.log(10.0)))
    out = O.maxvol_select(info, score, k, scale, 3, 5)
    assert len(out) == k and np.all(np.diff(out) > 0)  # pool order
