"""The composed device front end (pipeline.FrontEnd) against the oracle chain.

Each stage of one step is run on the device for B streams, its inputs and
outputs are snapshotted, and the oracle runs the same stage on the same
inputs: keypoint/match indices and information blocks bit-exact, poses within
1e-5 relative (north_star), the active-matching claims and RNG-driven pool
identical. This is what makes the bench step a valid measurement of the
reference path rather than of a look-alike.
"""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
from gf_orb_slam_amd import synth
from gf_orb_slam_amd.matcher import MAP_POINT_DTYPE, MP_VIEW_DTYPE
from gf_orb_slam_amd.orb import KEYPOINT_DTYPE

pytestmark = pytest.mark.gpu
B = 3


def _kp(t, b, n):
    return t[b].cpu().numpy().view(KEYPOINT_DTYPE).reshape(-1)[:n].copy()


def _pose_edges(kps, kp2mp, mps, invs):
    idx = np.nonzero(kp2mp >= 0)[0]
    return idx, mps["pos"][kp2mp[idx]], np.c_[kps["x"][idx], kps["y"][idx]], invs[kps["octave"][idx]]


def _check_pose(fe, b, T0, kps, kp2mp_before, mps, Tg, outl_g, ninl_g):
    idx, X, z, invs = _pose_edges(kps, kp2mp_before, mps, fe.inv_sigma2)
    To, oo, no, _ = O.pose_opt(T0, X, z, np.arange(len(idx), dtype=np.int32), invs, *fe.cam[2:])
    assert ninl_g == no
    assert np.array_equal(outl_g[idx], oo)
    assert np.all(np.abs(Tg.reshape(4, 4).astype(np.float64) - To) <= 1e-5 * np.maximum(1, np.abs(To)))


@pytest.fixture(scope="module")
def fe():
    from gf_orb_slam_amd.pipeline import FrontEnd

    fe = FrontEnd("euroc", 1000, B, 2000, seed=3)
    w, h = fe.cam[:2]
    fe.load_frames(np.stack([synth.synth_frame(w, h, synth.frame_seed(40 + b, 0)) for b in range(B)]))
    fe.build_maps()
    return fe


def test_pipeline_stages_match_oracle(fe):
    import torch

    s = fe.stream
    with torch.cuda.stream(s):
        fe.extract()
        fe.predict_pose()
        fe.reset_matches()
        fe.match_last_frame()
    fe.sync()
    nk = fe.nkp.cpu().numpy()
    T_pred = fe.Tcw.cpu().numpy()
    mps = fe.mps.cpu().numpy().view(MAP_POINT_DTYPE).reshape(B, -1)
    mdesc = fe.mp_desc.cpu().numpy()
    last_kp2mp = fe.last_kp2mp.cpu().numpy()
    last_pos = fe.last_pos.cpu().numpy()
    kp2mp_m3 = fe.kp2mp.cpu().numpy().copy()
    score_m3 = fe.score.cpu().numpy().copy()
    kps = [_kp(fe.kps, b, nk[b]) for b in range(B)]
    desc = [fe.desc[b, :nk[b]].cpu().numpy() for b in range(B)]
    for b in range(B):
        # M3: SearchByProjection(CurrentFrame, LastFrame, 15), checkOri
        k2 = np.full(nk[b], -1, np.int32)
        sc = np.full(nk[b], 999, np.int32)
        O.match_lastframe(fe.info, kps[b], desc[b], T_pred[b].reshape(4, 4), kps[b], desc[b],
                          last_kp2mp[b, :nk[b]].copy(), np.zeros(nk[b], np.uint8), last_pos[b, :nk[b]], 15.0, 1,
                          k2, sc)
        assert np.array_equal(k2, kp2mp_m3[b, :nk[b]]) and np.array_equal(sc, score_m3[b, :nk[b]])
        assert (k2 >= 0).sum() >= 20  # TrackWithMotionModel needs >= 20 (Tracking.cc:1541)

    with torch.cuda.stream(s):
        fe.pose_optimization(0)
    fe.sync()
    T1 = fe.Tcw.cpu().numpy()
    outl = fe.outl.cpu().numpy()
    ninl = fe.ninl.cpu().numpy()
    for b in range(B):
        _check_pose(fe, b, T_pred[b], kps[b], kp2mp_m3[b, :nk[b]], mps[b], T1[b], outl[b, :nk[b]], ninl[b])

    with torch.cuda.stream(s):
        fe.discard_outliers()
        fe.frame_info()
        fe.frustum()
        fe.map_info()
    fe.sync()
    kp2mp_d = fe.kp2mp.cpu().numpy().copy()
    nmatch = fe.nmatch.cpu().numpy()
    ntm = fe.num_to_match.cpu().numpy()
    Xv = fe.Xv.cpu().numpy()
    base = fe.base.cpu().numpy()
    f_info = fe.f_info.cpu().numpy()
    m_n = fe.m_n.cpu().numpy()
    views = fe.views.cpu().numpy().view(MP_VIEW_DTYPE).reshape(B, -1)
    map_info = fe.mp_info.cpu().numpy()
    map_H = fe.mp_H.cpu().numpy()
    map_uv = fe.mp_uv.cpu().numpy()
    map_valid = fe.mp_valid.cpu().numpy()
    score_d = fe.score.cpu().numpy().copy()
    for b in range(B):
        k = kp2mp_m3[b, :nk[b]].copy()
        k[outl[b, :nk[b]] == 1] = -1
        assert np.array_equal(k, kp2mp_d[b, :nk[b]])
        assert nmatch[b] == (k >= 0).sum() and ntm[b] == fe.budget - nmatch[b]
        # G1 on the device vs the host port
        Twc = np.eye(4, dtype=np.float32)
        T = T1[b].reshape(4, 4)
        Twc[:3, :3] = T[:3, :3].T
        Twc[:3, 3] = ((-T[0, :3] * T[0, 3]) + (-T[1, :3] * T[1, 3])) + (-T[2, :3] * T[2, 3])
        xv = O.obs_update(0.0, np.eye(4, dtype=np.float32), 1.0 / fe.fps, Twc)
        np.testing.assert_allclose(Xv[b], xv, rtol=1e-12, atol=1e-12)
        # FRAME_INFO_MATRIX over the matched points, in keypoint order
        idx = np.nonzero(k >= 0)[0]
        assert m_n[b] == len(idx)
        pos = mps[b]["pos"][k[idx]]
        s2 = fe.level_sigma2[kps[b]["octave"][idx]]
        H, info, uv, valid = O.obs_build_info(fe.obs_cam, Xv[b], pos, s2, 0)
        assert np.array_equal(info, f_info[b, :len(idx)])
        acc = np.eye(7).reshape(-1) * 1e-5
        for j in range(len(idx)):
            if valid[j]:
                acc = acc + info[j]
        np.testing.assert_allclose(base[b], acc, rtol=1e-12, atol=1e-15)
        # isInFrustum + exclusion of matched points
        v, _ = O.frustum(fe.info, T, mps[b])
        v["in_view"][k[idx]] = 0
        assert np.array_equal(v, views[b])
        # MAP_INFO_MATRIX
        H2, info2, uv2, valid2 = O.obs_build_info(fe.obs_cam, Xv[b], mps[b]["pos"], None, 0)
        assert np.array_equal(info2, map_info[b]) and np.array_equal(H2, map_H[b].reshape(-1, 14))
        assert np.array_equal(valid2, map_valid[b])

    with torch.cuda.stream(s):
        fe.active_match()
    fe.sync()
    kp2mp_a = fe.kp2mp.cpu().numpy()
    score_a = fe.score.cpu().numpy()
    n_act = fe.n_active.cpu().numpy()
    for b in range(B):
        k2 = kp2mp_d[b, :nk[b]].copy()
        sc = score_d[b, :nk[b]].copy()
        seed = 1 + fe.seed * 1000 + b
        nm, left = O.active_match(fe.info, kps[b], desc[b], views[b], mdesc[b], map_valid[b], map_info[b],
                                  map_H[b].reshape(-1, 14), map_uv[b].reshape(-1, 2), base[b], fe.level_sigma2,
                                  int(ntm[b]), 1.0, 0.8, seed, k2, sc)
        assert nm == n_act[b]
        assert np.array_equal(k2, kp2mp_a[b, :nk[b]])
        assert np.array_equal(sc, score_a[b, :nk[b]])
        assert nm > 0

    with torch.cuda.stream(s):
        fe.pose_optimization(1)
        fe.discard_outliers()
    fe.sync()
    T2 = fe.Tcw.cpu().numpy()
    outl2 = fe.outl.cpu().numpy()
    ninl2 = fe.ninl.cpu().numpy()
    for b in range(B):
        _check_pose(fe, b, T1[b], kps[b], kp2mp_a[b, :nk[b]], mps[b], T2[b], outl2[b, :nk[b]], ninl2[b])
        # the synthetic map was built from the identity camera: the pose is recovered
        assert np.abs(T2[b].reshape(4, 4) - np.eye(4)).max() < 2e-2


def test_pipeline_step_repeatable(fe):
    """A full step is deterministic given the RNG state."""
    import torch

    fe.rng.copy_(fe.rng0)
    fe.step()
    fe.sync()
    a = (fe.Tcw.cpu().numpy().copy(), fe.kp2mp.cpu().numpy().copy())
    fe.rng.copy_(fe.rng0)
    fe.step()
    fe.sync()
    assert np.array_equal(a[0], fe.Tcw.cpu().numpy()) and np.array_equal(a[1], fe.kp2mp.cpu().numpy())
    del torch
