"""Track-loss paths of the tracking step (csrc/reloc.hip) against the CPU
oracle: the matchers of TrackPreviousFrame (ORBmatcher::WindowSearch,
SearchByProjection(F1, F2, window)) and of Relocalisation
(SearchByProjection(F, KF, found, th, ORBdist), DetectRelocalisationCandidates)
one problem at a time, then the front end on sequences that lose track:
blank frames (no keypoints: TrackWithMotionModel and TrackPreviousFrame fail,
the stream goes LOST and relocalises against its keyframe database when
images return) and a jump along the loop (the motion model misses,
TrackPreviousFrame takes over). Every step is compared field by field with
the oracle chain, copied-in and free-running, as test_pipeline_gpu does.
Parity is against the oracle's restatement (no fixture of the reference
covers these paths: parity unpinned, docs/ORACLE_ASSUMPTIONS.md A20)."""
import numpy as np
import pytest

import oracle_chain as C
import oracle_lib as O
from gf_orb_slam_amd import reloc, scene, synth
from gf_orb_slam_amd.bow import FeatureVector
from gf_orb_slam_amd.matcher import MAP_POINT_DTYPE, FrameInfo
from gf_orb_slam_amd.orb import KEYPOINT_DTYPE
from gf_orb_slam_amd.pipeline import RELOC_KF_DTYPE, STATS, TR, KeyframeDB

pytestmark = pytest.mark.gpu

INFO = FrameInfo.make(752, 480, 458.654, 457.296, 367.215, 248.375)


def _project(T, X):
    Pc = X @ T[:3, :3].T + T[:3, 3]
    return INFO.fx * Pc[:, 0] / Pc[:, 2] + INFO.cx, INFO.fy * Pc[:, 1] / Pc[:, 2] + INFO.cy


def _pose(rx, ry, tx, ty, tz):
    cx, sx, cy, sy = np.cos(rx), np.sin(rx), np.cos(ry), np.sin(ry)
    R = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]]) @ np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = (tx, ty, tz)
    return T.astype(np.float32)


def _two_frames(seed, n=700, noise=10, dup=0.05):
    """A scene of n points seen from two nearby poses: F1 (last frame, map
    point ids, 15% NULL) and F2 (current frame: the visible points with
    descriptor noise, angles jittered, 10% clutter); some duplicated F2
    descriptors make distance ties."""
    rng = np.random.default_rng(seed)
    X = np.stack([rng.uniform(-4, 4, n), rng.uniform(-2.5, 2.5, n), rng.uniform(2.5, 9, n)], 1).astype(np.float32)
    T1, T2 = _pose(0, 0, 0, 0, 0), _pose(0.01, -0.02, 0.05, -0.02, 0.03)
    u1, v1 = _project(T1.astype(np.float64), X.astype(np.float64))
    u2, v2 = _project(T2.astype(np.float64), X.astype(np.float64))
    vis = (u1 > 1) & (u1 < 750) & (v1 > 1) & (v1 < 478) & (u2 > 1) & (u2 < 750) & (v2 > 1) & (v2 < 478)
    X, u1, v1, u2, v2 = X[vis], u1[vis], v1[vis], u2[vis], v2[vis]
    m = len(X)
    oct_ = rng.integers(0, 8, m)
    K1 = np.zeros(m, KEYPOINT_DTYPE)
    K1["x"], K1["y"], K1["octave"], K1["angle"] = u1, v1, oct_, rng.uniform(0, 360, m)
    D1 = rng.integers(0, 256, (m, 32), dtype=np.uint8)
    mp1 = rng.permutation(4000)[:m].astype(np.int32)
    mp1[rng.uniform(size=m) < 0.15] = -1
    nc = m // 10
    K2 = np.zeros(m + nc, KEYPOINT_DTYPE)
    K2["x"][:m] = u2 + rng.normal(0, 0.7, m)
    K2["y"][:m] = v2 + rng.normal(0, 0.7, m)
    K2["octave"][:m] = oct_
    K2["angle"][:m] = (K1["angle"] + rng.normal(0, 4, m)) % 360
    K2["x"][m:], K2["y"][m:] = rng.uniform(0, 751, nc), rng.uniform(0, 479, nc)
    K2["octave"][m:], K2["angle"][m:] = rng.integers(0, 8, nc), rng.uniform(0, 360, nc)
    D2 = np.concatenate([synth.flip_bits(rng, D1, noise), rng.integers(0, 256, (nc, 32), dtype=np.uint8)])
    nd = int(dup * len(D2))
    a, b = rng.integers(0, len(D2), nd), rng.integers(0, len(D2), nd)
    D2[a] = D2[b]
    perm = rng.permutation(len(K2))  # keypoint order unrelated to F1's
    return dict(X=X, T1=T1, T2=T2, K1=K1, D1=D1, mp1=mp1, K2=K2[perm], D2=D2[perm])


@pytest.mark.parametrize("seed,window,min_level", [(1, 200, 4), (2, 100, 0), (3, 15, 0), (4, 50, 2)])
def test_window_search_matches_oracle(seed, window, min_level):
    F = _two_frames(seed)
    args = (F["K2"], F["D2"], F["K1"], F["D1"], F["mp1"], window, min_level)
    n_d, out_d = reloc.window_search(INFO, *args)
    n_o, out_o = O.window_search(INFO, *args)
    assert n_d == n_o and np.array_equal(out_d, out_o), (n_d, n_o)
    assert n_d > 10


@pytest.mark.parametrize("seed,window", [(5, 15), (6, 50), (7, 3)])
def test_search_frames_matches_oracle(seed, window):
    F = _two_frames(seed)
    rng = np.random.default_rng(seed)
    n2 = len(F["K2"])
    kp2mp = np.full(n2, -1, np.int32)  # some matches already set (spMapPointsAlreadyFound)
    pre = rng.choice(n2, n2 // 8, replace=False)
    kp2mp[pre] = rng.choice(F["mp1"][F["mp1"] >= 0], len(pre), replace=False)
    score = np.full(n2, 999, np.int32)
    pos1 = F["X"][:len(F["K1"])]
    args = (F["K2"], F["D2"], F["T2"], F["K1"], F["D1"], F["mp1"], pos1, window, kp2mp, score)
    n_d, km_d, sc_d = reloc.search_frames(INFO, *args)
    n_o, km_o, sc_o = O.search_frames(INFO, *args)
    assert n_d == n_o and np.array_equal(km_d, km_o) and np.array_equal(sc_d, sc_o), (n_d, n_o)
    assert n_d > 0


@pytest.mark.parametrize("seed,th,orb_dist", [(8, 10.0, 100), (9, 3.0, 64)])
def test_search_kf_projection_matches_oracle(seed, th, orb_dist):
    F = _two_frames(seed)
    rng = np.random.default_rng(seed)
    m = len(F["X"])
    mps = np.zeros(4000, MAP_POINT_DTYPE)
    mp_desc = rng.integers(0, 256, (4000, 32), dtype=np.uint8)
    ids = F["mp1"]
    ok = ids >= 0
    mps["pos"][ids[ok]] = F["X"][ok]
    d = np.linalg.norm(F["X"][ok].astype(np.float64), axis=1).astype(np.float32)
    mps["min_dist"][ids[ok]] = d / rng.uniform(1.0, 3.0, ok.sum()).astype(np.float32)
    mps["max_dist"][ids[ok]] = d * 4
    mp_desc[ids[ok]] = F["D1"][ok]
    found = (rng.uniform(size=4000) < 0.2).astype(np.uint8)
    n2 = len(F["K2"])
    kp2mp = np.full(n2, -1, np.int32)
    kp2mp[rng.choice(n2, n2 // 10, replace=False)] = np.flatnonzero(found)[:n2 // 10]
    score = np.full(n2, 999, np.int32)
    args = (F["K2"], F["D2"], F["T2"], F["K1"], ids, mps, mp_desc, found, th, orb_dist, kp2mp, score)
    n_d, km_d, sc_d = reloc.search_kf_projection(INFO, *args)
    n_o, km_o, sc_o = O.search_kf_projection(INFO, *args)
    assert n_d == n_o and np.array_equal(km_d, km_o) and np.array_equal(sc_d, sc_o), (n_d, n_o)
    assert n_d > 10
    del m


def _oracle_transform(voc):
    def t(d):
        w, v, (nodes, start, feats) = O.bow_transform(voc, d, 4)
        return w, v, FeatureVector(nodes, start, feats)
    return t


def test_reloc_candidates_match_oracle():
    """DetectRelocalisationCandidates over a chain of queries: keyframes of
    overlapping descriptor sets, queries mixing two keyframes' descriptors with
    noise; the keyframes' query state carries over (stale scores of unscored
    keyframes enter the covisibility sums)."""
    rng = np.random.default_rng(21)
    voc = synth.synth_vocabulary_fast(11, k=10, L=5)
    pool = rng.integers(0, 256, (3000, 32), dtype=np.uint8)
    nkf = 12
    kf_desc, kf_kps = [], []
    for k in range(nkf):
        idx = (np.arange(400) + 200 * k) % 3000
        kf_desc.append(synth.flip_bits(rng, pool[idx], 6))
        kp = np.zeros(400, KEYPOINT_DTYPE)
        kp["x"], kp["y"] = rng.uniform(0, 751, 400), rng.uniform(0, 479, 400)
        kf_kps.append(kp)
    db = KeyframeDB(kf_kps, kf_desc, _oracle_transform(voc))
    cov = [[j for j in (k - 1, k + 1, k - 2, k + 2) if 0 <= j < nkf] for k in range(nkf)]
    cov_off = np.concatenate([[0], np.cumsum([len(c) for c in cov])]).astype(np.int32)
    cov_flat = np.array([j for c in cov for j in c], np.int32)
    bad = np.zeros(nkf, np.uint8)
    bad[7] = 1
    st_d = np.zeros(64, RELOC_KF_DTYPE)
    st_o = np.zeros(64, RELOC_KF_DTYPE)
    total = 0
    for q in range(1, 9):
        a, b = rng.integers(0, nkf, 2)
        d = np.concatenate([synth.flip_bits(rng, kf_desc[a][:250], 8), synth.flip_bits(rng, kf_desc[b][:150], 8)])
        w, v, _ = O.bow_transform(voc, d, 4)
        c_d = reloc.reloc_candidates(w, v, db, bad, cov_off, cov_flat, q, st_d)
        c_o = O.reloc_candidates(w, v, db, bad, cov_off, cov_flat, q, st_o)
        assert np.array_equal(c_d, c_o), (q, c_d, c_o)
        assert np.array_equal(st_d, st_o), q
        total += len(c_d)
    assert total > 0


# ---------------------------------------------------------------- the step
def _scene_setup(B, G, seed, voc, blank=(), jump=(), n_kf=24):
    """Keyframe-graph streams with their databases; frames of scene s at
    indices `blank` (pairs (s, idx)) are uniform grey, and (s, idx, src)
    in `jump` replace a frame with the image at another loop index."""
    import torch

    from gf_orb_slam_amd.bow import ORBVocabulary
    from gf_orb_slam_amd.pipeline import FrontEnd

    W = scene.Workload("euroc", B, n_scenes=min(B, 3), period=32, seed=seed)
    frames = W.render_all("cuda").contiguous()
    for s, i in blank:
        frames[s, i] = 100
    src = frames.clone()
    for s, i, j in jump:
        frames[s, i] = src[s, j]
    gmaps = W.build_global_maps(lambda im: O.extract(im), G, n_kf=n_kf)
    dvoc = ORBVocabulary(voc)
    dbs = [KeyframeDB(gm["kf_kps"], gm["kf_desc"], dvoc.transform) for gm in gmaps]
    fe = FrontEnd("euroc", 1000, B, G, 100)
    fe.set_vocab(dvoc)
    T, V = W.boot_state()
    for b in range(B):
        gm = gmaps[W.scene_of[b]]
        fe.set_map(b, gm["mp"], gm["desc"])
        fe.set_covis(b, gm["graph"])
        fe.set_kfdb(b, dbs[W.scene_of[b]])
        fe.set_rng(b, 7 + b)
    fe.set_source(frames, W.scene_of, W.phase)
    fe.bootstrap(T, V, 0.0)
    torch.cuda.synchronize()
    return W, frames.cpu().numpy(), gmaps, dbs, fe, T, V, dvoc


def _chain(gm, db, voc, G):
    ch = C.Chain("euroc", 1000, G, 100)
    ch.set_map(gm["mp"], gm["desc"])
    ch.set_covis(gm["graph"])
    ch.set_kfdb(db)
    ch.set_vocab(voc)
    return ch


EXACT = ["kps", "desc", "nkp", "kp2mp", "score", "outlier", "last_kps", "last_desc", "last_nkp", "last_kp2mp",
         "last_outlier", "last_pos", "views", "mp_upd", "rng", "t_prev", "t_cur", "track", "reloc"]


def _compare(dev, ch, b, prefix):
    n = int(ch.read("nkp"))
    for k in EXACT:
        a, o = dev[k][b], ch.read(k)
        if k in ("kps", "desc"):  # a frame with fewer keypoints leaves the device buffer's tail as it was
            a, o = a[:n], o[:n]
        assert np.array_equal(a, o), f"{prefix}{k} differs (stream {b})"
    nl = int(ch.stats()["nleft"])
    assert np.array_equal(dev["left"][b][:nl], ch.read("left")[:nl]), f"{prefix}leftovers differ (stream {b})"
    for k in ("Tcw", "velocity", "Tcw_last"):
        a, o = dev[k][b].astype(np.float64), ch.read(k).astype(np.float64)
        assert np.all(np.abs(a - o) <= 1e-5 * np.maximum(1, np.abs(o))), f"{prefix}{k} differs (stream {b})"
    for k in ("Xv", "Xv_next", "base", "mp_H", "mp_info", "mp_uv"):
        np.testing.assert_allclose(dev[k][b], ch.read(k), rtol=1e-9, atol=1e-12, err_msg=f"{prefix}{k} (stream {b})")
    sd, so = dev["stats"][:, b], ch.read("stats")
    assert np.array_equal(sd, so), f"{prefix}stage counters differ (stream {b}): " + str(
        {STATS[i]: (int(sd[i]), int(so[i])) for i in range(len(STATS)) if sd[i] != so[i]})


def _run(W, fr, gmaps, dbs, fe, T, V, voc, G, nsteps):
    B = fe.B
    free = []
    for b in range(B):
        s = W.scene_of[b]
        ch = _chain(gmaps[s], dbs[s], voc, G)
        ch.set_rng(7 + b)
        ch.bootstrap(fr[s, W.phase[b] % W.period], T[b], V[b])
        free.append(ch)
    dev = C.read_state(fe)
    log = []
    for k in range(1, nsteps + 1):
        before = dev
        fe.step()
        dev = C.read_state(fe)
        for b in range(B):
            s = W.scene_of[b]
            img = fr[s, (W.phase[b] + k) % W.period]
            ch = _chain(gmaps[s], dbs[s], voc, G)
            ch.load_from(before, b)
            ch.write("reloc", before["reloc"][b])  # set_kfdb reset it
            ch.step(img)
            _compare(dev, ch, b, f"step {k}: ")
            free[b].step(img)
            _compare(dev, free[b], b, f"free-running step {k}: ")
            st = {n: int(dev["stats"][i, b]) for i, n in enumerate(STATS)}
            log.append((k, b, int(dev["track"][b][TR["path"]]), int(dev["track"][b][TR["ok"]]),
                        int(dev["track"][b][TR["state"]]), st["flags"], st["tpf"], st["ncand"], st["reloc"],
                        st["ransac"], st["inl2"]))
    return log


def test_lost_and_relocalised():
    """Blank frames: the stream loses track (TrackPreviousFrame finds nothing),
    stays LOST while the frames are blank (no BoW words, no candidates), then
    relocalises against its keyframe database; the two frames after run
    TrackPreviousFrame and th 5. Device and oracle agree on every field."""
    B, G = 3, 2600
    voc = synth.synth_vocabulary_fast(11, k=10, L=5)
    W0 = scene.Workload("euroc", B, n_scenes=3, period=32, seed=4)
    blank = [(W0.scene_of[b], (W0.phase[b] + k) % 32) for b in range(B) for k in (3, 4)]
    setup = _scene_setup(B, G, 4, voc, blank=blank)
    W, fr, gmaps, dbs, fe, T, V, dvoc = setup
    log = _run(W, fr, gmaps, dbs, fe, T, V, voc, G, 10)
    for row in log:
        print(row)
    paths = [r[2] for r in log]
    assert paths.count(3) >= B and paths.count(2) >= B, paths  # relocalisation, then TrackPreviousFrame
    assert any(r[5] & 32768 for r in log), "no stream relocalised"
    assert any(r[9] > 0 for r in log), "no RANSAC iteration ran"
    fe.close()


def test_motion_model_miss_falls_back_to_previous_frame():
    """A jump of 4 frames along the loop: the constant-velocity prediction
    misses, TrackPreviousFrame (or the relocalisation after it) takes over."""
    B, G = 3, 2600
    voc = synth.synth_vocabulary_fast(11, k=10, L=5)
    W0 = scene.Workload("euroc", B, n_scenes=3, period=32, seed=5)
    jump = [(W0.scene_of[b], (W0.phase[b] + k) % 32, (W0.phase[b] + k + 4) % 32) for b in range(B) for k in (5,)]
    W, fr, gmaps, dbs, fe, T, V, dvoc = _scene_setup(B, G, 5, voc, jump=jump)
    log = _run(W, fr, gmaps, dbs, fe, T, V, voc, G, 9)
    for row in log:
        print(row)
    assert any(r[2] in (1, 2) for r in log), "TrackPreviousFrame never ran"
    fe.close()


def test_lost_after_database_detached():
    """A stream relocalises (blank frames 3-4), then its keyframe graph is set
    again (gf_frontend_set_covis detaches the keyframe database) and it loses
    track a second time (blank frames 9-10): with no database the stream stays
    LOST, and no relocalisation may reuse the first loss's candidates (they
    index the detached database). Free-running and copied-in against the oracle
    chain, whose database is detached at the same step."""
    B, G = 3, 2600
    voc = synth.synth_vocabulary_fast(11, k=10, L=5)
    W0 = scene.Workload("euroc", B, n_scenes=3, period=32, seed=4)
    blank = [(W0.scene_of[b], (W0.phase[b] + k) % 32) for b in range(B) for k in (3, 4, 9, 10)]
    W, fr, gmaps, dbs, fe, T, V, dvoc = _scene_setup(B, G, 4, voc, blank=blank)
    free = []
    for b in range(B):
        s = W.scene_of[b]
        ch = _chain(gmaps[s], dbs[s], voc, G)
        ch.set_rng(7 + b)
        ch.bootstrap(fr[s, W.phase[b] % W.period], T[b], V[b])
        free.append(ch)
    dev = C.read_state(fe)
    detach_after = 7
    relocalised, lost_late = 0, 0
    for k in range(1, 13):
        if k == detach_after + 1:
            for b in range(B):
                fe.set_covis(b, gmaps[W.scene_of[b]]["graph"])
                free[b].set_covis(gmaps[W.scene_of[b]]["graph"])
                free[b].set_kfdb(None)
            dev = C.read_state(fe)
        before = dev
        fe.step()
        dev = C.read_state(fe)
        for b in range(B):
            s = W.scene_of[b]
            img = fr[s, (W.phase[b] + k) % W.period]
            ch = _chain(gmaps[s], dbs[s] if k <= detach_after else None, voc, G)
            ch.load_from(before, b)
            ch.write("reloc", before["reloc"][b])
            ch.step(img)
            _compare(dev, ch, b, f"step {k}: ")
            free[b].step(img)
            _compare(dev, free[b], b, f"free-running step {k}: ")
            st = {n: int(dev["stats"][i, b]) for i, n in enumerate(STATS)}
            if k <= detach_after and st["flags"] & 32768:
                relocalised += 1
            if k > detach_after:
                assert not st["flags"] & 32768, f"step {k}: stream {b} relocalised without a database"
                lost_late += int(dev["track"][b][TR["state"]] == 1)
    assert relocalised > 0, "no stream relocalised before the database was detached"
    assert lost_late > 0, "no stream lost track after the database was detached"
    fe.close()


def test_few_keyframes_track_previous_frame():
    """A keyframe graph of 3 keyframes: mpMap->KeyFramesInMap() < 4 sends the
    initial estimate to TrackPreviousFrame every frame, velocity or not
    (Tracking.cc:602); device and oracle chain agree on every field."""
    B, G = 2, 2600
    voc = synth.synth_vocabulary_fast(11, k=10, L=5)
    W, fr, gmaps, dbs, fe, T, V, dvoc = _scene_setup(B, G, 6, voc, n_kf=3)
    log = _run(W, fr, gmaps, dbs, fe, T, V, voc, G, 5)
    paths = [r[2] for r in log]
    assert all(p in (2, 3) for p in paths), paths  # never the motion model (3: relocalisation after a loss)
    assert paths.count(2) >= len(paths) // 2, paths
    fe.close()
