"""The composed device front end (pipeline.FrontEnd) against the oracle chain.

After one warm-up step (so the map carries observability state stamped by the
previous frame's prediction pass), every stage of the next step runs on the
device for B streams; its inputs and outputs are snapshotted and the oracle
runs the same stage on the same inputs (tests/oracle_chain.py): keypoint and
match indices, information blocks and frame stamps bit-exact, poses within
1e-5 relative (north_star), active-matching claims identical. This is what
makes the bench step a measurement of the reference path and not of a
look-alike.
"""
import numpy as np
import pytest

import oracle_chain as C
import oracle_lib as O
from gf_orb_slam_amd import synth
from gf_orb_slam_amd.matcher import MAP_POINT_DTYPE, MP_VIEW_DTYPE
from gf_orb_slam_amd.orb import KEYPOINT_DTYPE

B = 3


def _np(t):
    return t.cpu().numpy().copy()


def _kp(t, b, n):
    return t[b].cpu().numpy().view(KEYPOINT_DTYPE).reshape(-1)[:n].copy()


class _P:  # the oracle_chain.Prepared fields the stage helpers read
    pass


def _prep(fe, mps_b):
    P = _P()
    P.obs_cam, P.level_sigma2, P.mps, P.info = fe.obs_cam, fe.level_sigma2, mps_b, fe.info
    return P


def _state(fe, b):
    st = C.MapState(fe.M)
    st.H = _np(fe.mp_H[b]).reshape(-1, 14)
    st.info = _np(fe.mp_info[b]).reshape(-1, 49)
    st.uv = _np(fe.mp_uv[b]).reshape(-1, 2)
    st.upd = _np(fe.mp_upd[b]).astype(np.int64)
    return st


def _same_state(fe, b, st):
    assert np.array_equal(_np(fe.mp_upd[b]), st.upd)
    assert np.array_equal(_np(fe.mp_info[b]).reshape(-1, 49), st.info)
    assert np.array_equal(_np(fe.mp_H[b]).reshape(-1, 14), st.H)
    assert np.array_equal(_np(fe.mp_uv[b]).reshape(-1, 2), st.uv)


def _check_pose(fe, T0, kps, kp2mp_before, mps, Tg, outl_g, ninl_g):
    idx = np.nonzero(kp2mp_before >= 0)[0]
    To, oo, no, _ = O.pose_opt(T0, mps["pos"][kp2mp_before[idx]], np.c_[kps["x"][idx], kps["y"][idx]],
                               kps["octave"][idx].astype(np.int32), fe.inv_sigma2, *fe.cam[2:])
    assert ninl_g == no
    assert np.array_equal(outl_g[idx], oo)
    assert np.all(np.abs(Tg.reshape(4, 4).astype(np.float64) - To) <= 1e-5 * np.maximum(1, np.abs(To)))


# config 2 (EuRoC 752x480, 1000 feats, GF budget 100, 2000-point map) and
# config 3 (TUM 640x480, 2000 feats, GF budget 160, 3000-point map)
@pytest.fixture(scope="module", params=[("euroc", 1000, 2000, 100), ("tum", 2000, 3000, 160)],
                ids=["config2", "config3"])
def fe(request):
    from gf_orb_slam_amd.pipeline import FrontEnd

    cam, nfeat, nmap, budget = request.param
    fe = FrontEnd(cam, nfeat, B, nmap, gf_budget=budget, seed=3)
    w, h = fe.cam[:2]
    fe.load_frames(np.stack([synth.synth_frame(w, h, synth.frame_seed(40 + b, 0)) for b in range(B)]))
    fe.build_maps()
    return fe


@pytest.mark.gpu
def test_pipeline_stages_match_oracle(fe):
    import torch

    fe.reset_state()
    fe.step()  # warm: leaves next-frame stamps in the map
    fe.sync()
    fid = fe.frame_id
    states = [_state(fe, b) for b in range(B)]
    assert all((s.upd == fid).sum() > 100 for s in states)  # predicted-visible points carry the stamp

    s = fe.stream
    with torch.cuda.stream(s):
        fe.extract()
        fe.predict_pose()
        fe.reset_matches()
        fe.match_last_frame()
    fe.sync()
    nk = _np(fe.nkp)
    T_pred = _np(fe.Tcw)
    mps = fe.mps.cpu().numpy().view(MAP_POINT_DTYPE).reshape(B, -1)
    mdesc = _np(fe.mp_desc)
    last_kp2mp, last_pos = _np(fe.last_kp2mp), _np(fe.last_pos)
    kp2mp_m3, score_m3 = _np(fe.kp2mp), _np(fe.score)
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
    T1, outl, ninl = _np(fe.Tcw), _np(fe.outl), _np(fe.ninl)
    for b in range(B):
        _check_pose(fe, T_pred[b], kps[b], kp2mp_m3[b, :nk[b]], mps[b], T1[b], outl[b, :nk[b]], ninl[b])

    with torch.cuda.stream(s):
        fe.discard_outliers()
        fe.frame_info()
        fe.frustum()
        fe.map_info()
    fe.sync()
    kp2mp_d, score_d = _np(fe.kp2mp), _np(fe.score)
    nmatch, ntm = _np(fe.nmatch), _np(fe.num_to_match)
    Xv, base = _np(fe.Xv), _np(fe.base)
    views = fe.views.cpu().numpy().view(MP_VIEW_DTYPE).reshape(B, -1)
    updated = _np(fe.mp_updated)
    for b in range(B):
        k = kp2mp_m3[b, :nk[b]].copy()
        k[outl[b, :nk[b]] == 1] = -1
        assert np.array_equal(k, kp2mp_d[b, :nk[b]])
        assert nmatch[b] == (k >= 0).sum() and ntm[b] == fe.budget - nmatch[b]
        T = T1[b].reshape(4, 4)
        xv = O.obs_update(0.0, np.eye(4, dtype=np.float32), 1.0 / fe.fps, C.twc_of(T))
        np.testing.assert_allclose(Xv[b], xv, rtol=1e-12, atol=1e-12)
        P, st = _prep(fe, mps[b]), states[b]
        C.frame_info_stage(P, Xv[b], kps[b], k, np.zeros(nk[b], np.uint8), st)
        acc = C.accumulate_stage(k, st, fid)
        np.testing.assert_allclose(base[b], acc, rtol=1e-13, atol=1e-18)
        assert np.abs(acc - np.eye(7).reshape(-1) * 1e-5).max() > 0  # stamped matches contribute
        v, _ = O.frustum(fe.info, T, mps[b])
        v["in_view"][k[k >= 0]] = 0
        assert np.array_equal(v, views[b])
        upd = C.map_info_stage(P, Xv[b], v, 0, st, fid)
        assert np.array_equal(upd, updated[b])
        _same_state(fe, b, st)

    fe.rng.copy_(fe.rng0)
    with torch.cuda.stream(s):
        fe.active_match()
    fe.sync()
    kp2mp_a, score_a, n_act = _np(fe.kp2mp), _np(fe.score), _np(fe.n_active)
    for b in range(B):
        k2 = kp2mp_d[b, :nk[b]].copy()
        sc = score_d[b, :nk[b]].copy()
        st = states[b]
        nm, _ = O.active_match(fe.info, kps[b], desc[b], views[b], mdesc[b], updated[b], st.info, st.H, st.uv,
                               base[b], fe.level_sigma2, int(ntm[b]), 1.0, 0.8, 1 + fe.seed * 1000 + b, k2, sc)
        assert nm == n_act[b] and nm > 0
        assert np.array_equal(k2, kp2mp_a[b, :nk[b]])
        assert np.array_equal(sc, score_a[b, :nk[b]])

    with torch.cuda.stream(s):
        fe.pose_optimization(1)
        fe.discard_outliers()
        fe.predict_next()
    fe.sync()
    T2, outl2, ninl2 = _np(fe.Tcw), _np(fe.outl), _np(fe.ninl)
    Xv2, Xn = _np(fe.Xv), _np(fe.Xv_next)
    for b in range(B):
        _check_pose(fe, T1[b], kps[b], kp2mp_a[b, :nk[b]], mps[b], T2[b], outl2[b, :nk[b]], ninl2[b])
        assert np.abs(T2[b].reshape(4, 4) - np.eye(4)).max() < 2e-2  # map built from the identity camera
        xv = O.obs_update(0.0, np.eye(4, dtype=np.float32), 1.0 / fe.fps, C.twc_of(T2[b].reshape(4, 4)))
        np.testing.assert_allclose(Xv2[b], xv, rtol=1e-12, atol=1e-12)
        xn = np.array(O.obs_predict(Xv2[b], 1.0 / fe.fps, 2)[1].Xv)
        np.testing.assert_allclose(Xn[b], xn, rtol=1e-12, atol=1e-13)
        st = states[b]
        C.map_info_stage(_prep(fe, mps[b]), Xn[b], None, 1, st, fid + 1)
        _same_state(fe, b, st)


@pytest.mark.gpu
def test_pipeline_step_repeatable(fe):
    """A full step is deterministic given the RNG state and the map stamps."""
    fe.reset_state()
    fe.step()
    fe.step()
    fe.sync()
    a = (_np(fe.Tcw), _np(fe.kp2mp), _np(fe.mp_info))
    fe.reset_state()
    fe.step()
    fe.step()
    fe.sync()
    assert np.array_equal(a[0], _np(fe.Tcw)) and np.array_equal(a[1], _np(fe.kp2mp))
    assert np.array_equal(a[2], _np(fe.mp_info))


def test_oracle_chain_tracks_pose():
    """CPU chain sanity (also what bench.py times as cpu_baseline)."""
    P = C.prepare("euroc", 1000, synth.synth_frame(752, 480, synth.frame_seed(77, 0)), 7)
    r1 = C.step(P)
    r2 = C.step(P)
    for r in (r1, r2):
        assert r["ninliers"] >= 80 and r["n_active"] > 0
        assert np.abs(r["Tcw"] - np.eye(4)).max() < 2e-2
    assert (P.state.upd == P.fid).sum() > 100
