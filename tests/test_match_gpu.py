"""GPU parity of frustum culling (M7) and projection matching (M2, M3) with
the sequential CPU oracle: identical kp->map-point claims, scores, counts."""
import numpy as np
import pytest

import oracle_lib as O
from gf_orb_slam_amd import synth
from gf_orb_slam_amd.matcher import Frame, FrameInfo, ORBmatcher

pytestmark = pytest.mark.gpu


def _scene(cam, nmp, nkp, seed, **kw):
    sc = synth.synth_scene(cam, nmp, nkp, seed, **kw)
    return sc, FrameInfo.make(*sc["camera"])


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_frustum_bit_exact(seed):
    sc, info = _scene("euroc", 3000, 1000, seed)
    F = Frame(sc["keypoints"], sc["descriptors"], info, sc["Tcw"])
    vg = F.isInFrustum(sc["map"], 0.5)
    vo, n = O.frustum(info, sc["Tcw"], sc["map"])
    assert vg.tobytes() == vo.tobytes()
    assert vg["in_view"].sum() == n


@pytest.mark.parametrize("cam,nmp,nkp,seed,th,ratio", [
    ("euroc", 2000, 1000, 1, 1.0, 0.8),    # local-map search, Tracking.cc:3323
    ("euroc", 2000, 1000, 2, 5.0, 0.8),    # after relocalisation (th = 5), large windows, many conflicts
    ("tum", 3000, 2000, 3, 1.0, 0.8),
    ("tum", 3000, 2000, 4, 3.0, 0.6),      # default th / nnratio
    ("euroc", 500, 3000, 5, 10.0, 0.9),    # dense distractors, long claim chains
])
def test_search_by_projection_bit_exact(cam, nmp, nkp, seed, th, ratio):
    sc, info = _scene(cam, nmp, nkp, seed)
    F = Frame(sc["keypoints"], sc["descriptors"], info, sc["Tcw"])
    views = F.isInFrustum(sc["map"], 0.5)
    # pre-claim a few keypoints (matches from the motion-model stage)
    rng = np.random.default_rng(seed)
    pre = rng.choice(nkp, nkp // 20, replace=False)
    F.mvpMapPoints[pre] = 100000 + pre
    F.mvpMatchScore[pre] = 7
    kp2mp, score = F.mvpMapPoints.copy(), F.mvpMatchScore.copy()
    ng = ORBmatcher(ratio).SearchByProjection(F, views, sc["mp_desc"], th)
    no = O.match_project(info, sc["keypoints"], sc["descriptors"], views, sc["mp_desc"], th, ratio, kp2mp, score)
    assert ng == no
    np.testing.assert_array_equal(F.mvpMapPoints, kp2mp)
    np.testing.assert_array_equal(F.mvpMatchScore, score)
    assert ng > 0


def test_search_by_projection_budget():
    """M5 (ORBmatcher.cc:276-379): the M2 search with IncreaseFound; a
    non-positive budget matches nothing, a positive one runs the full list."""
    sc, info = _scene("euroc", 2000, 1000, 9)
    F = Frame(sc["keypoints"], sc["descriptors"], info, sc["Tcw"])
    views = F.isInFrustum(sc["map"], 0.5)
    assert ORBmatcher(0.8).SearchByProjection_Budget(F, views, sc["mp_desc"], 1.0, 0.0) == 0
    assert (F.mvpMapPoints < 0).all()
    kp2mp, score = F.mvpMapPoints.copy(), F.mvpMatchScore.copy()
    found = np.zeros(len(views), np.int32)
    ng = ORBmatcher(0.8).SearchByProjection_Budget(F, views, sc["mp_desc"], 1.0, 5.0, found)
    no = O.match_project(info, sc["keypoints"], sc["descriptors"], views, sc["mp_desc"], 1.0, 0.8, kp2mp, score)
    assert ng == no and np.array_equal(F.mvpMapPoints, kp2mp) and np.array_equal(F.mvpMatchScore, score)
    expect = np.zeros(len(views), np.int32)
    np.add.at(expect, kp2mp[kp2mp >= 0], 1)
    assert np.array_equal(found, expect) and found.sum() == ng


def _two_frames(seed, nmp=2500, nkp=1500, rot_deg=0.3):
    sc, info = _scene("euroc", nmp, nkp, seed)
    rng = np.random.default_rng(seed + 100)
    last = Frame(sc["keypoints"], sc["descriptors"], info, sc["Tcw"])
    last.mvpMapPoints[:] = sc["kp_mp"]
    ok = sc["kp_mp"] >= 0
    last.mp_pos[ok] = sc["map"]["pos"][sc["kp_mp"][ok]]
    last.mvbOutlier[rng.choice(nkp, nkp // 15, replace=False)] = 1
    # current frame: same map seen from a slightly moved camera
    T = sc["Tcw"].astype(np.float64).copy()
    d = synth.look_pose(rng, 0.01, rot_deg).astype(np.float64)
    Tc = (d @ T).astype(np.float32)
    X = sc["map"]["pos"].astype(np.float64)
    u, v, z = synth.project(Tc, X, sc["camera"])
    kps = sc["keypoints"].copy()
    m = sc["kp_mp"]
    kps["x"][ok] = np.clip(u[m[ok]] + rng.uniform(-1, 1, ok.sum()), 0, 751)
    kps["y"][ok] = np.clip(v[m[ok]] + rng.uniform(-1, 1, ok.sum()), 0, 479)
    kps["angle"] = (kps["angle"] + 4.0 + rng.normal(0, 3, nkp)) % 360
    desc = synth.flip_bits(rng, sc["descriptors"], 10)
    cur = Frame(kps, desc, info, Tc)
    return last, cur, info


@pytest.mark.parametrize("seed,th,ori", [(1, 15.0, True), (2, 15.0, False), (3, 45.0, True), (4, 7.0, True)])
def test_search_by_projection_lastframe_bit_exact(seed, th, ori):
    last, cur, info = _two_frames(seed)
    kp2mp, score = cur.mvpMapPoints.copy(), cur.mvpMatchScore.copy()
    ng = ORBmatcher(0.9, ori).SearchByProjectionLast(cur, last, th)
    no = O.match_lastframe(info, cur.mvKeysUn, cur.mDescriptors, cur.mTcw, last.mvKeysUn, last.mDescriptors,
                           last.mvpMapPoints, last.mvbOutlier, last.mp_pos, th, ori, kp2mp, score)
    assert ng == no and ng > 100
    np.testing.assert_array_equal(cur.mvpMapPoints, kp2mp)
    np.testing.assert_array_equal(cur.mvpMatchScore, score)


def test_descriptor_distance_gpu():
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (1000, 32), dtype=np.uint8)
    b = rng.integers(0, 256, (1000, 32), dtype=np.uint8)
    d = ORBmatcher.DescriptorDistance(a, b)
    ref = np.unpackbits(a ^ b, axis=1).sum(1)
    np.testing.assert_array_equal(d, ref)


def test_empty_inputs():
    sc, info = _scene("euroc", 10, 20, 9)
    F = Frame(sc["keypoints"][:0], sc["descriptors"][:0], info, sc["Tcw"])
    assert ORBmatcher().SearchByProjection(F, np.zeros(0, dtype=F.isInFrustum(sc["map"]).dtype),
                                           np.zeros((0, 32), np.uint8)) == 0
