"""The C++ drop-in layer (include/gfslam/orbslam.h) driven the way Tracking
drives the reference classes (tests/cpp/dropin_frontend.cpp), compared with
the CPU oracle: keypoints/descriptors and match indices bit-exact, pose within
1e-5 relative, outlier flags and active-matching claims identical; then
ComputeBoW, both SearchByBoW overloads, SearchByProjection_OnePoint,
SearchByProjection_Budget and setSelction_Number through the same layer."""
import os
import subprocess

import numpy as np
import pytest

import oracle_lib as O
from gf_orb_slam_amd import synth
from gf_orb_slam_amd.matcher import FrameInfo
from gf_orb_slam_amd.observability import ObsCamera
from gf_orb_slam_amd.optimizer import inv_level_sigma2
from gf_orb_slam_amd.orb import KEYPOINT_DTYPE

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "cpp", "dropin_frontend")


def test_dropin_binary_built():
    assert os.path.exists(BIN), "run make (or __graft_entry__.build())"


@pytest.mark.gpu
def test_dropin_frontend_matches_oracle(tmp_path):
    cam = synth.CAMERAS["euroc"]
    w, h, fx, fy, cx, cy = cam
    img = synth.synth_frame(w, h, synth.frame_seed(3, 7))
    k, d = O.extract(img)
    rng = np.random.default_rng(12)
    mps, mdesc = synth.build_local_map(k, d, cam, rng, 1500)
    T0 = synth.look_pose(rng, 0.005, 0.2)
    with open(tmp_path / "params.txt", "w") as f:
        f.write(f"{w} {h} {fx} {fy} {cx} {cy} {len(mps)}\n" + " ".join(repr(float(x)) for x in T0.reshape(-1)))
    img.tofile(tmp_path / "img.u8")
    rec = np.zeros((len(mps), 64), np.uint8)
    rec[:, :32] = mps.view(np.uint8).reshape(-1, 32)
    rec[:, 32:] = mdesc
    rec.tofile(tmp_path / "map.bin")
    voc = synth.synth_vocabulary(7, k=10, L=3)
    synth.write_vocab_binary(voc, str(tmp_path / "voc.bin"))
    r = subprocess.run([BIN, str(tmp_path)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    N, nview, nm, ninl, N2, n3, nact, dd = map(int, open(tmp_path / "summary.txt").read().split())
    rd = lambda name, dt: np.fromfile(tmp_path / name, dt)

    # extraction (E1-E8)
    kg = rd("kps.bin", KEYPOINT_DTYPE)
    assert N == len(k) and kg.tobytes() == k.tobytes()
    assert np.array_equal(rd("desc.bin", np.uint8).reshape(-1, 32), d)
    assert dd == int(np.unpackbits(d[0] ^ d[1]).sum())

    # isInFrustum + SearchByProjection(F, local, 1), nnratio 0.8 (M7, M2)
    info = FrameInfo.make(*cam)
    views, nv = O.frustum(info, T0, mps)
    assert nv == nview
    k2 = np.full(N, -1, np.int32)
    sc = np.full(N, 999, np.int32)
    no = O.match_project(info, k, d, views, mdesc, 1.0, 0.8, k2, sc)
    assert no == nm and np.array_equal(k2, rd("kp2mp_m2.i32", np.int32))

    # PoseOptimization (P1-P4)
    idx = np.nonzero(k2 >= 0)[0]
    To, oo, no_, _ = O.pose_opt(T0, mps["pos"][k2[idx]], np.c_[k["x"][idx], k["y"][idx]],
                                k["octave"][idx].astype(np.int32), inv_level_sigma2(), fx, fy, cx, cy)
    Tg = rd("pose.f32", np.float32).reshape(4, 4)
    assert ninl == no_
    assert np.all(np.abs(Tg.astype(np.float64) - To) <= 1e-5 * np.maximum(1, np.abs(To)))
    og = rd("outl.u8", np.uint8)
    assert np.array_equal(og[idx], oo) and og[k2 < 0].sum() == 0

    # SearchByProjection(Cur, Last, 15) with the rotation check (M3)
    pos = np.zeros((N, 3), np.float32)
    pos[idx] = mps["pos"][k2[idx]]
    k3 = np.full(N, -1, np.int32)
    s3 = np.full(N, 999, np.int32)
    n3o = O.match_lastframe(info, k, d, Tg, k, d, k2.copy(), og.copy(), pos, 15.0, 1, k3, s3)
    assert N2 == N and n3o == n3 and np.array_equal(k3, rd("kp2mp_m3.i32", np.int32))

    # Observability: PWLS state, MAP_INFO_MATRIX, runActiveMapMatching (G1-G7)
    Twc = np.eye(4, dtype=np.float32)
    Twc[:3, :3] = Tg[:3, :3].T
    Twc[:3, 3] = ((-Tg[0, :3] * Tg[0, 3]) + (-Tg[1, :3] * Tg[1, 3])) + (-Tg[2, :3] * Tg[2, 3])
    xv = O.obs_update(0.0, Tg, 0.05, Twc)
    assert np.array_equal(xv, rd("xv.f64", np.float64))
    v2, _ = O.frustum(info, Tg, mps)
    v2["in_view"][k3[k3 >= 0]] = 0
    ocam = ObsCamera.for_tracking(fx, fy, cx, cy, w, h)
    H, inf, uv, valid = O.obs_build_info(ocam, xv, mps["pos"], None, 0)
    upd = ((v2["in_view"] != 0) & (valid != 0)).astype(np.uint8)
    sig2 = (info.scale_factors() ** 2).astype(np.float32)
    ka = k3.copy()
    nao, _ = O.active_match(info, k, d, v2, mdesc, upd, inf, H, uv, np.eye(7).reshape(-1) * 1e-5, sig2, 40, 1.0,
                            0.8, 5, ka, s3.copy())
    assert nao == nact and nact > 0
    assert np.array_equal(ka, rd("kp2mp_act.i32", np.int32))

    nb0, nb1, p0, one, nbud0, found, nbud, no_time, ok = map(int, open(tmp_path / "summary2.txt").read().split())
    # Frame::ComputeBoW (D1): transform(levelsup 4)
    from gf_orb_slam_amd.bow import read_vocabulary
    vtree = read_vocabulary(str(tmp_path / "voc.bin"))  # the file's float weights, as the loader reads them
    words, values, fv = O.bow_transform(vtree, d, 4)
    assert np.array_equal(rd("bow_words.i32", np.int32), words)
    assert np.array_equal(rd("bow_values.f64", np.float64), values)
    for name, o in zip(("fv_nodes", "fv_start", "fv_feats"), fv):
        assert np.array_equal(rd(name + ".i32", np.int32), o), name
    # SearchByBoW(KeyFrame, Frame) and SearchByBoW(KeyFrame, KeyFrame), nnratio 0.75 with the
    # rotation check (M6): KF = F with its M2 claims, F2 = the same image, KF2 = F2 after active matching
    n0, o0 = O.match_bow(0, 0.75, True, (fv, d, k, k2), (fv, d, k, np.full(N, -1, np.int32)))
    assert n0 == nb0 and n0 > 0 and np.array_equal(o0, rd("bow_kf_f.i32", np.int32))
    n1, o1 = O.match_bow(1, 0.75, True, (fv, d, k, k2), (fv, d, k, ka))
    assert n1 == nb1 and n1 > 0 and np.array_equal(o1, rd("bow_kf_kf.i32", np.int32))
    # SearchByProjection_OnePoint (M4) of F's first matched map point, then
    # SearchByProjection_Budget (M5, th 0.8) over the whole local map on a fresh frame
    assert p0 == k2[np.nonzero(k2 >= 0)[0][0]]
    v3, _ = O.frustum(info, Tg, mps)
    only = v3.copy()
    only["in_view"][:] = 0
    only["in_view"][p0] = v3["in_view"][p0]
    kp3 = np.full(N, -1, np.int32)
    sc3 = np.full(N, 999, np.int32)
    O.match_project(info, k, d, only, mdesc, 1.0, 0.8, kp3, sc3)
    hit = np.nonzero(kp3 == p0)[0]
    assert one == (int(hit[0]) if len(hit) else -1) and one >= 0
    assert nbud0 == 0  # time_constr <= 0 returns at once (ORBmatcher.cc:281-282)
    nb = O.match_project(info, k, d, v3, mdesc, 0.8, 0.8, kp3, sc3)
    assert nb == nbud and found == nbud
    assert np.array_equal(kp3, rd("budget_kp2mp.i32", np.int32)) and np.array_equal(sc3, rd("budget_score.i32", np.int32))
    # Observability::setSelction_Number(300, 3, ...) over the local map at kinematic[1] (G7)
    import ctypes
    from gf_orb_slam_amd.observability import Rng
    # the driver's Observability gets the camera as the float K[] it read (Observability(fu, fv, ...) takes doubles)
    ocam = ObsCamera.for_tracking(*(float(np.float32(v)) for v in (fx, fy, cx, cy)), w, h)
    ks = O.obs_predict(xv, 0.05, 2)
    xv1 = np.array(ks[1].Xv[:])
    # batchInfoMat_Map (:556-644) over the local list: every 7th point was
    # updated this frame (its own block, score 0.5), every 11th too with score
    # -1; the others are rebuilt at kinematic[1], visible ones into the pool
    # (score 1, stamped), invisible ones get score -1 (stamp unchanged)
    pos = np.ascontiguousarray(mps["pos"], np.float32)
    n = len(pos)
    _, blk_all, _, valid = O.obs_build_info(ocam, xv1, pos, None, 1)
    blk_all = blk_all.reshape(n, 49)
    pre = np.array([i % 7 == 3 for i in range(n)])
    pre_neg = np.array([(i % 7 != 3) and (i % 11 == 4) for i in range(n)])
    fresh = ~pre & ~pre_neg
    score = np.where(pre, 0.5, np.where(pre_neg, -1.0, np.where(valid.astype(bool), 1.0, -1.0)))
    pool = np.nonzero(score >= 0)[0]
    pinfo = np.ascontiguousarray(np.where(pre[pool, None], 0.0, blk_all[pool]))
    for j, i in enumerate(pool):
        if pre[i]:
            pinfo[j, [0, 8, 16, 24, 32, 40, 48]] = 1e3 * (1 + (i % 5))
    pscore = np.ascontiguousarray(score[pool])
    sel = np.zeros(len(pool), np.int32)
    nsel = ctypes.c_int()
    assert O.orc().orc_select_pool(O._p(pinfo), O._p(pscore), len(pool), 300, 3, 8, ctypes.byref(Rng.seeded(9)),
                                   O._p(sel), ctypes.byref(nsel)) == 0
    assert no_time == 0 and ok == 1
    gsel = rd("select.i32", np.int32)
    assert len(gsel) == nsel.value == 300 and np.array_equal(gsel, pool[sel[:nsel.value]])
    np.testing.assert_allclose(rd("select_blocks.f64", np.float64).reshape(-1, 49), pinfo[sel[:nsel.value]],
                               rtol=1e-9, atol=1e-12)
    assert np.array_equal(rd("select_scores.f64", np.float64), score)
    stamps = rd("select_stamps.i32", np.int32)
    assert (stamps[pre | pre_neg] == 5).all() and (stamps[fresh & valid.astype(bool)] == 5).all()
    assert (stamps[fresh & ~valid.astype(bool)] != 5).all()


SEQ_BIN = os.path.join(ROOT, "tests", "cpp", "sequence_driver")


def test_sequence_driver_built():
    assert os.path.exists(SEQ_BIN), "run make (or __graft_entry__.build())"


@pytest.mark.gpu
def test_cpp_sequence_and_local_ba_through_the_abi(tmp_path):
    """tests/cpp/sequence_driver: a C++ program that only links libgfslam
    tracks two rendered sequences for 7 frames (bootstrap + steps from host
    frames) and runs LocalBundleAdjustment(pKF, &mbAbortBA) free and stopped;
    every step equals the CPU oracle chain running free, the local BA results
    equal the oracle (iterations capped at (0, 0) for the stopped call: the flag is raised before the solve)."""
    import oracle_chain as C
    from gf_orb_slam_amd import scene

    B, F, M, nfeat, budget = 2, 8, 1500, 1000, 100
    W = scene.Workload("euroc", B, n_scenes=2, period=32, seed=6, tex_size=256)
    fr = W.render_all("cpu").numpy()
    maps = W.build_maps(lambda im: O.extract(im), M)
    T, V = W.boot_state()
    w, h, fx, fy, cx, cy = W.cam
    frames = np.stack([np.stack([fr[W.scene_of[b], (W.phase[b] + k) % W.period] for b in range(B)])
                       for k in range(F)])
    frames.tofile(tmp_path / "frames.u8")
    mp = np.zeros((B, M), maps[0][0].dtype)
    md = np.zeros((B, M, 32), np.uint8)
    nmp = np.zeros(B, np.int32)
    for b in range(B):
        m, d = maps[W.scene_of[b]]
        mp[b, :len(m)], md[b, :len(m)], nmp[b] = m, d, len(m)
    mp.tofile(tmp_path / "maps.bin")
    md.tofile(tmp_path / "maps_desc.bin")
    nmp.tofile(tmp_path / "nmp.i32")
    np.concatenate([T.reshape(-1), V.reshape(-1)]).astype(np.float32).tofile(tmp_path / "boot.f32")
    with open(tmp_path / "params.txt", "w") as f:
        f.write(f"{w} {h} {fx} {fy} {cx} {cy} {nfeat} {B} {M} {budget} {F}\n")
    p = synth.synth_lba_problem(21, 12, 1500)
    np.array([len(p["kf_kind"]), len(p["pt_pos"]), len(p["edge_pt"])], np.int32).tofile(tmp_path / "ba_sizes.i32")
    for k, name in (("kf_Tcw", "kf_Tcw"), ("kf_kind", "kf_kind"), ("kf_cam", "kf_cam"), ("pt_pos", "pt_pos"),
                    ("edge_pt", "edge_pt"), ("edge_kf", "edge_kf"), ("edge_z", "edge_z"),
                    ("edge_inv_sigma2", "edge_is2")):
        np.ascontiguousarray(p[k]).tofile(tmp_path / f"ba_{name}.bin")
    r = subprocess.run([SEQ_BIN, str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr

    chains = []
    for b in range(B):
        ch = C.Chain("euroc", nfeat, M, budget)
        ch.set_map(*maps[W.scene_of[b]])
        ch.set_rng(1 + b)
        ch.bootstrap(frames[0, b], T[b], V[b])
        chains.append(ch)
    cap = chains[0].cap
    kp2mp = np.fromfile(tmp_path / "seq_kp2mp.i32", np.int32).reshape(F - 1, B, cap)
    tcw = np.fromfile(tmp_path / "seq_tcw.f32", np.float32).reshape(F - 1, B, 16)
    for k in range(1, F):
        for b in range(B):
            chains[b].step(frames[k, b])
            assert np.array_equal(kp2mp[k - 1, b], chains[b].read("kp2mp")), (k, b)
            To = chains[b].read("Tcw").astype(np.float64)
            assert np.all(np.abs(tcw[k - 1, b] - To) <= 1e-5 * np.maximum(1, np.abs(To))), (k, b)

    def _lba(tag):
        nkf, npts = len(p["kf_kind"]), len(p["pt_pos"])
        return (np.fromfile(tmp_path / f"lba_{tag}_T.f32", np.float32).reshape(nkf, 4, 4),
                np.fromfile(tmp_path / f"lba_{tag}_X.f32", np.float32).reshape(npts, 3),
                np.fromfile(tmp_path / f"lba_{tag}_out.u8", np.uint8),
                np.fromfile(tmp_path / f"lba_{tag}_it.i32", np.int32))

    for tag, its in (("free", (5, 10)), ("stop", (0, 0))):
        Tg, Xg, og, ig = _lba(tag)
        To, Xo, oo, io = O.local_ba(p, its=its)
        assert list(ig) == list(io) and np.array_equal(og, oo), tag
        assert np.all(np.abs(Tg - To) <= 1e-5 * np.maximum(1, np.abs(To))), tag
        assert np.all(np.abs(Xg - Xo) <= 1e-5 * np.maximum(1, np.abs(Xo))), tag
