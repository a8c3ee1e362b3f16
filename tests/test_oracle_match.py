"""Oracle checks for the matching rows (M1-M3, M7), no GPU."""
import ctypes

import numpy as np

import oracle_lib as O
from gf_orb_slam_amd import synth
from gf_orb_slam_amd.matcher import FrameInfo


def test_descriptor_distance_is_popcount():
    rng = np.random.default_rng(0)
    a = rng.integers(0, 256, (200, 32), dtype=np.uint8)
    b = rng.integers(0, 256, (200, 32), dtype=np.uint8)
    f = O.orc().orc_descriptor_distance
    for i in range(200):
        ref = int(np.unpackbits(a[i] ^ b[i]).sum())
        assert f(ctypes.c_void_p(a[i].ctypes.data), ctypes.c_void_p(b[i].ctypes.data)) == ref


def test_project_matches_ground_truth():
    sc = synth.synth_scene("euroc", 2000, 1000, 11)
    info = FrameInfo.make(*sc["camera"])
    views, nv = O.frustum(info, sc["Tcw"], sc["map"])
    assert nv > 500
    kp2mp = np.full(1000, -1, np.int32)
    score = np.full(1000, 999, np.int32)
    n = O.match_project(info, sc["keypoints"], sc["descriptors"], views, sc["mp_desc"], 1.0, 0.8, kp2mp, score)
    ok = kp2mp >= 0
    assert n == ok.sum() > 400
    assert (kp2mp[ok] == sc["kp_mp"][ok]).mean() > 0.98
    assert np.all(score[ok] <= 100) and np.all(score[~ok] == 999)


def test_lastframe_histogram_range():
    """Rotation bins are round(rot/30) so only bins 0..12 can be hit
    (kept)."""
    rot = np.arange(0, 360, 0.25, dtype=np.float32)
    bins = np.round(rot * np.float32(1.0 / 30)).astype(int)
    bins[bins == 30] = 0
    assert bins.max() == 12
