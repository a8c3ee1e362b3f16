"""ctypes loader of the CPU oracle (oracle/liboracle.so) — test infrastructure.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline use this.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from gf_orb_slam_amd.orb import KEYPOINT_DTYPE

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_PATH = os.path.join(ROOT, "oracle", "liboracle.so")
_orc = None


def orc() -> ctypes.CDLL:
    global _orc
    if _orc is None:
        _orc = ctypes.CDLL(os.environ.get("GF_ORACLE_LIB", ORACLE_PATH))
        _orc.orc_fast_atan2.restype = ctypes.c_float
        _orc.orc_fast_atan2.argtypes = [ctypes.c_float, ctypes.c_float]
    return _orc


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def extract(img: np.ndarray, nfeatures=1000, scale=1.2, nlevels=8, fast_th=20, score_type=1):
    """ORBextractor(nfeatures, scale, nlevels, score_type, fast_th)(img): score_type
    1 FAST_SCORE, 0 HARRIS_SCORE (ORBextractor.h:57)."""
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    cap = nfeatures + 64
    kps = np.zeros(cap, KEYPOINT_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n = ctypes.c_int()
    rc = orc().orc_extract_st(_p(img), w, h, w, nfeatures, ctypes.c_float(scale), nlevels, score_type, fast_th,
                              _p(kps), _p(desc), cap, ctypes.byref(n))
    assert rc == 0, rc
    return kps[:n.value].copy(), desc[:n.value].copy()


def level(img: np.ndarray, lvl: int, which: int, nfeatures=1000, scale=1.2, nlevels=8):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    lw, lh = ctypes.c_int(), ctypes.c_int()
    orc().orc_extract_level(_p(img), w, h, nfeatures, ctypes.c_float(scale), nlevels, lvl, which, None,
                            ctypes.byref(lw), ctypes.byref(lh))
    out = np.zeros((lh.value, lw.value), np.uint8)
    orc().orc_extract_level(_p(img), w, h, nfeatures, ctypes.c_float(scale), nlevels, lvl, which, _p(out),
                            ctypes.byref(lw), ctypes.byref(lh))
    return out


def plan(w, h, nfeatures=1000, scale=1.2, nlevels=8):
    lw = np.zeros(nlevels, np.int32)
    lh = np.zeros(nlevels, np.int32)
    fpl = np.zeros(nlevels, np.int32)
    sc = np.zeros(nlevels, np.float32)
    um = np.zeros(16, np.int32)
    orc().orc_extractor_plan(w, h, nfeatures, ctypes.c_float(scale), nlevels, _p(lw), _p(lh), _p(fpl), _p(sc),
                             _p(um))
    return lw, lh, fpl, sc, um


def frustum(info, Tcw, mps, view_cos=0.5):
    from gf_orb_slam_amd.matcher import MP_VIEW_DTYPE
    mps = np.ascontiguousarray(mps)
    views = np.zeros(len(mps), MP_VIEW_DTYPE)
    n = ctypes.c_int()
    orc().orc_frustum(ctypes.byref(info), _p(np.ascontiguousarray(Tcw, np.float32)), _p(mps), len(mps),
                      ctypes.c_float(view_cos), _p(views), ctypes.byref(n))
    return views, n.value


def match_project(info, kps, desc, views, mp_desc, th, nnratio, kp2mp, score):
    n = ctypes.c_int()
    orc().orc_match_project(ctypes.byref(info), _p(kps), _p(desc), len(kps), _p(views), _p(mp_desc), len(views),
                            ctypes.c_float(th), ctypes.c_float(nnratio), _p(kp2mp), _p(score), ctypes.byref(n))
    return n.value


def match_lastframe(info, kps, desc, Tcw, last_kps, last_desc, last_kp2mp, last_outlier, last_pos, th, check_ori,
                    kp2mp, score):
    n = ctypes.c_int()
    orc().orc_match_lastframe(ctypes.byref(info), _p(kps), _p(desc), len(kps),
                              _p(np.ascontiguousarray(Tcw, np.float32)), _p(last_kps), _p(last_desc),
                              _p(last_kp2mp), _p(last_outlier), _p(np.ascontiguousarray(last_pos, np.float32)),
                              len(last_kps), ctypes.c_float(th), int(check_ori), _p(kp2mp), _p(score),
                              ctypes.byref(n))
    return n.value


# ----------------------------------------------------------------- GF (G1-G7)
class Kine(ctypes.Structure):
    _fields_ = [("dt", ctypes.c_double), ("dt_inseg", ctypes.c_double), ("Xv", ctypes.c_double * 13),
                ("F_Q", ctypes.c_double * 16), ("F_Omg", ctypes.c_double * 12), ("F_Q_inSeg", ctypes.c_double * 16),
                ("F_Omg_inSeg", ctypes.c_double * 12), ("Tcw", ctypes.c_float * 16)]


def obs_predict(Xv, dt, nseg):
    out = (Kine * nseg)()
    xv = np.ascontiguousarray(Xv, np.float64)
    orc().orc_obs_predict(_p(xv), ctypes.c_double(dt), nseg, out)
    return list(out)


def obs_update(t0, Tcw0, t1, Twc1):
    xv = np.zeros(13)
    orc().orc_obs_update(ctypes.c_double(t0), _p(np.ascontiguousarray(Tcw0, np.float32)), ctypes.c_double(t1),
                         _p(np.ascontiguousarray(Twc1, np.float32)), _p(xv))
    return xv


def obs_build_info(cam, Xv, pos, sigma2, check_viz):
    pos = np.ascontiguousarray(pos, np.float32)
    n = len(pos)
    H = np.zeros((n, 14))
    info = np.zeros((n, 49))
    uv = np.zeros((n, 2), np.float32)
    valid = np.zeros(n, np.uint8)
    s2 = None if sigma2 is None else np.ascontiguousarray(sigma2, np.float32)
    orc().orc_obs_build_info(ctypes.byref(cam), _p(np.ascontiguousarray(Xv, np.float64)), _p(pos), _p(s2), n,
                             int(check_viz), _p(H), _p(info), _p(uv), _p(valid))
    return H, info, uv, valid


def logdet(M):
    M = np.ascontiguousarray(M, np.float64).reshape(-1, 49)
    out = np.zeros(len(M))
    orc().orc_logdet(_p(M), len(M), _p(out))
    return out


def rand_sequence(seed, n):
    out = np.zeros(n, np.int32)
    orc().orc_rand_sequence(ctypes.c_uint(seed), n, _p(out))
    return out


def active_match(info_fi, kps, desc, views, mp_desc, updated, info, H, uv, base, level_sigma2, num_to_match, th,
                 nnratio, seed, kp2mp, score):
    m = len(views)
    left = np.zeros(m, np.int32)
    nleft, nmatched = ctypes.c_int(), ctypes.c_int()
    orc().orc_obs_active_match(ctypes.byref(info_fi), _p(kps), _p(desc), len(kps), _p(views), _p(mp_desc),
                               _p(np.ascontiguousarray(updated, np.uint8)), _p(np.ascontiguousarray(info)),
                               _p(np.ascontiguousarray(H)), _p(np.ascontiguousarray(uv, np.float32)), m,
                               _p(np.ascontiguousarray(base, np.float64)),
                               _p(np.ascontiguousarray(level_sigma2, np.float32)), num_to_match, ctypes.c_float(th),
                               ctypes.c_float(nnratio), ctypes.c_uint(seed), _p(kp2mp), _p(score), _p(left),
                               ctypes.byref(nleft), ctypes.byref(nmatched))
    return nmatched.value, left[:nleft.value].copy()


def last_rand_calls():
    """std::rand() calls made by the last active_match / maxvol_select."""
    return orc().orc_last_rand_calls()


def maxvol_select(info, score, k, sample_scale, mode, seed):
    info = np.ascontiguousarray(info, np.float64).reshape(-1, 49)
    n = len(info)
    out = np.zeros(n, np.int32)
    nout = ctypes.c_int()
    orc().orc_maxvol_select(_p(info), _p(np.ascontiguousarray(score, np.float64)), n, k, ctypes.c_double(sample_scale),
                            mode, ctypes.c_uint(seed), _p(out), ctypes.byref(nout))
    return out[:nout.value].copy()


def pose_opt(Tcw, X, z, octave, inv_sigma2, fx, fy, cx, cy):
    """Optimizer::PoseOptimization on the CPU oracle; returns (Tcw, outlier, ninliers, iterations)."""
    Tcw = np.ascontiguousarray(Tcw, np.float32).reshape(16)
    X = np.ascontiguousarray(X, np.float32).reshape(-1, 3)
    z = np.ascontiguousarray(z, np.float32).reshape(-1, 2)
    octave = np.ascontiguousarray(octave, np.int32)
    invs = np.ascontiguousarray(inv_sigma2, np.float32)
    n = len(X)
    out = np.zeros(16, np.float32)
    outl = np.zeros(max(n, 1), np.uint8)
    ninl, iters = ctypes.c_int(), ctypes.c_int()
    f = ctypes.c_float
    rc = orc().orc_pose_opt(_p(Tcw), _p(X), _p(z), _p(octave), _p(invs), n, f(fx), f(fy), f(cx), f(cy), _p(out),
                            _p(outl), ctypes.byref(ninl), ctypes.byref(iters))
    assert rc == 0, rc
    return out.reshape(4, 4), outl[:n].copy(), ninl.value, iters.value


def ldlt_solve(H, b):
    H = np.ascontiguousarray(H, np.float64).reshape(6, 6)
    b = np.ascontiguousarray(b, np.float64)
    x = np.zeros(6)
    ok = orc().orc_ldlt_solve(_p(H), _p(b), _p(x))
    return bool(ok), x


def local_ba(prob: dict, its=(5, 10)):
    """Optimizer::LocalBundleAdjustment on the CPU oracle; returns
    (kf_Tcw [nkf,4,4], pt_pos [npts,3], edge_outlier, iterations). `its` caps
    the two optimize() calls (a force stop = fewer iterations)."""
    from gf_orb_slam_amd.optimizer import BAArrays
    arr = BAArrays(prob)
    rc = orc().orc_local_ba_iters(ctypes.byref(arr.problem), ctypes.byref(arr.result), int(its[0]), int(its[1]))
    assert rc == 0, rc
    return arr.out()


def inverse3(m):
    m = np.ascontiguousarray(m, np.float64).reshape(9)
    r = np.zeros(9)
    orc().orc_inverse3(_p(m), _p(r))
    return r.reshape(3, 3)


def bow_transform(voc: dict, desc: np.ndarray, levelsup: int = 4):
    """TemplatedVocabulary::transform on the CPU oracle -> (words, values, (nodes, start, feats))."""
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    n = len(d)
    words, values = np.zeros(max(n, 1), np.int32), np.zeros(max(n, 1))
    nodes, start, feats = np.zeros(max(n, 1), np.int32), np.zeros(n + 1, np.int32), np.zeros(max(n, 1), np.int32)
    nw, nf = ctypes.c_int(), ctypes.c_int()
    t = {k: np.ascontiguousarray(voc[k], dt) for k, dt in (("parent", np.int32), ("desc", np.uint8),
                                                           ("weight", np.float64), ("is_leaf", np.uint8))}
    orc().orc_bow_transform(voc["k"], voc["L"], voc["scoring"], voc["weighting"], len(t["parent"]), _p(t["parent"]),
                            _p(t["desc"]), _p(t["weight"]), _p(t["is_leaf"]), _p(d), n, levelsup, _p(words),
                            _p(values), ctypes.byref(nw), _p(nodes), _p(start), _p(feats), ctypes.byref(nf))
    k = nf.value
    return words[:nw.value].copy(), values[:nw.value].copy(), (nodes[:k].copy(), start[:k + 1].copy(),
                                                                feats[:start[k]].copy())


def match_bow(mode, nnratio, check_ori, a, b):
    """ORBmatcher::SearchByBoW on the CPU oracle; a, b = ((nodes, start, feats), desc, kps, mp)."""
    def side(s):
        (nodes, start, feats), desc, kps, mp = s
        return [np.ascontiguousarray(nodes, np.int32), np.ascontiguousarray(start, np.int32),
                np.ascontiguousarray(feats, np.int32), np.ascontiguousarray(desc, np.uint8),
                np.ascontiguousarray(kps["angle"], np.float32), np.ascontiguousarray(mp, np.int32)]
    A, B = side(a), side(b)
    out = np.zeros(max(len(B[3]) if mode == 0 else len(A[3]), 1), np.int32)
    nm = ctypes.c_int()
    orc().orc_match_bow(mode, ctypes.c_float(nnratio), int(check_ori), _p(A[0]), _p(A[1]), _p(A[2]), len(A[0]),
                        _p(A[3]), _p(A[4]), _p(A[5]), len(A[3]), _p(B[0]), _p(B[1]), _p(B[2]), len(B[0]), _p(B[3]),
                        _p(B[4]), _p(B[5]), len(B[3]), _p(out), ctypes.byref(nm))
    return nm.value, out[:(len(B[3]) if mode == 0 else len(A[3]))].copy()


def undistort_keypoints(kps, K, dist):
    """Frame::UndistortKeyPoints on the CPU oracle (OpenCV undistortPoints restated)."""
    k = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    out = k.copy()
    Kf = np.asarray(K, np.float32).reshape(4)
    d = np.zeros(5, np.float32)
    d[:len(dist)] = np.asarray(dist, np.float32)
    assert orc().orc_undistort_keypoints(_p(Kf), _p(d), _p(k), len(k), _p(out)) == 0
    return out


def distinctive_descriptors(desc, offsets):
    """MapPoint::ComputeDistinctiveDescriptors on the CPU oracle: best row per point."""
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    off = np.ascontiguousarray(offsets, np.int32)
    nmp = len(off) - 1
    best = np.zeros(max(nmp, 1), np.int32)
    out = np.zeros((max(nmp, 1), 32), np.uint8)
    assert orc().orc_distinctive_descriptors(nmp, _p(d), _p(off), _p(best), _p(out)) == 0
    return best[:nmp], out[:nmp]


def fuse(info, Tcw, Ow, kps, desc, kf_mp, kf_mp_bad, mps, mp_desc, mp_skip, mp_ids, th):
    """ORBmatcher::Fuse on the CPU oracle: (nFused, results)."""
    from gf_orb_slam_amd.matcher import FUSE_RESULT_DTYPE, MAP_POINT_DTYPE
    kps = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    mps = np.ascontiguousarray(mps, MAP_POINT_DTYPE)
    res = np.zeros(len(mps), FUSE_RESULT_DTYPE)
    opt = lambda a, dt: None if a is None else np.ascontiguousarray(a, dt)
    n = ctypes.c_int()
    T, O = np.ascontiguousarray(Tcw, np.float32), np.ascontiguousarray(Ow, np.float32)
    args = [ctypes.byref(info), _p(T), _p(O), _p(kps), _p(np.ascontiguousarray(desc, np.uint8)), len(kps),
            _p(np.ascontiguousarray(kf_mp, np.int32)), _p(opt(kf_mp_bad, np.uint8)), _p(mps),
            _p(np.ascontiguousarray(mp_desc, np.uint8)), _p(opt(mp_skip, np.uint8)), _p(opt(mp_ids, np.int32)),
            len(mps), ctypes.c_float(th), _p(res), ctypes.byref(n)]
    assert orc().orc_fuse(*args) == 0
    return n.value, res


def search_triangulation(check_ori, a, b, F12, sigma2):
    """ORBmatcher::SearchForTriangulation on the CPU oracle: (n, vMatches12)."""
    def side(s):
        (nodes, start, feats), desc, kps, mp = s
        return [np.ascontiguousarray(nodes, np.int32), np.ascontiguousarray(start, np.int32),
                np.ascontiguousarray(feats, np.int32), np.ascontiguousarray(desc, np.uint8),
                np.ascontiguousarray(kps, KEYPOINT_DTYPE), np.ascontiguousarray(mp, np.int32)]
    A, B = side(a), side(b)
    out = np.zeros(max(len(A[3]), 1), np.int32)
    nm = ctypes.c_int()
    F = np.ascontiguousarray(F12, np.float32).reshape(9)
    s2 = np.ascontiguousarray(sigma2, np.float32)
    assert orc().orc_search_triangulation(int(check_ori), _p(A[0]), _p(A[1]), _p(A[2]), len(A[0]), _p(A[3]),
                                          _p(A[4]), _p(A[5]), len(A[3]), _p(B[0]), _p(B[1]), _p(B[2]), len(B[0]),
                                          _p(B[3]), _p(B[4]), _p(B[5]), len(B[3]), _p(F), _p(s2), _p(out),
                                          ctypes.byref(nm)) == 0
    return nm.value, out[:len(A[3])].copy()


def pnp_run(p3d, p2d, sigma2, K, params, seed, n_iter):
    """PnPsolver on the CPU oracle: std::srand(seed), then iterate(n_iter[c])
    for each c. Returns (Tcw [c,4,4], inliers [c,n], ninliers, flags, rand_calls)."""
    from gf_orb_slam_amd.pnp import PNP_PARAMS_DTYPE

    p3d = np.ascontiguousarray(p3d, np.float32).reshape(-1, 3)
    p2d = np.ascontiguousarray(p2d, np.float32).reshape(-1, 2)
    s2 = np.ascontiguousarray(sigma2, np.float32).reshape(-1)
    n = len(p3d)
    c = len(n_iter)
    it = np.ascontiguousarray(n_iter, np.int32)
    prm = np.ascontiguousarray(params, PNP_PARAMS_DTYPE).reshape(1)
    Kf = np.asarray(K, np.float32).reshape(4)
    T = np.zeros((c, 4, 4), np.float32)
    inl = np.zeros((c, max(n, 1)), np.uint8)
    ninl = np.zeros(c, np.int32)
    fl = np.zeros(c, np.int32)
    rc = np.zeros(c, np.int32)
    assert orc().orc_pnp_run(_p(p3d), _p(p2d), _p(s2), n, _p(Kf), _p(prm), ctypes.c_uint(seed), c, _p(it), _p(T),
                             _p(inl), _p(ninl), _p(fl), _p(rc)) == 0
    return T, inl[:, :n], ninl, fl, rc


def initialize(K, kps1, kps2, matches12, rng_state, sigma=1.0, iterations=200, min_triangulated=50):
    """Initializer::Initialize on the CPU oracle. rng_state (RNG_DTYPE [1]) is
    advanced in place. Returns (rc, result [1], p3d [n1,3], triangulated [n1])."""
    from gf_orb_slam_amd.initializer import INIT_RESULT_DTYPE
    k1 = np.ascontiguousarray(kps1, KEYPOINT_DTYPE)
    k2 = np.ascontiguousarray(kps2, KEYPOINT_DTYPE)
    m = np.ascontiguousarray(matches12, np.int32)
    Kf = np.ascontiguousarray(np.asarray(K, np.float32).reshape(9))
    res = np.zeros(1, INIT_RESULT_DTYPE)
    p3d = np.zeros((len(k1), 3), np.float32)
    tri = np.zeros(len(k1), np.uint8)
    f = orc().orc_initialize
    f.argtypes = [ctypes.c_void_p, ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_int,
                  ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                  ctypes.c_void_p]
    rc = f(_p(Kf), sigma, iterations, min_triangulated, _p(k1), len(k1), _p(k2), len(k2), _p(m), _p(rng_state),
           _p(res), _p(p3d), _p(tri))
    return rc, res, p3d, tri


def window_search(info, kps2, desc2, kps1, desc1, mp1, window, min_level, max_level=2**31 - 1, nnratio=0.9,
                  check_ori=True):
    """ORBmatcher::WindowSearch on the CPU oracle -> (nmatches, out[n2])."""
    k2, d2 = np.ascontiguousarray(kps2, KEYPOINT_DTYPE), np.ascontiguousarray(desc2, np.uint8)
    k1, d1 = np.ascontiguousarray(kps1, KEYPOINT_DTYPE), np.ascontiguousarray(desc1, np.uint8)
    m1 = np.ascontiguousarray(mp1, np.int32)
    out = np.zeros(max(len(k2), 1), np.int32)
    nm = ctypes.c_int()
    o = orc()
    o.orc_window_search(ctypes.byref(info), _p(k2), _p(d2), len(k2), _p(k1), _p(d1), _p(m1), len(k1), window,
                        min_level, max_level, ctypes.c_float(nnratio), int(check_ori), _p(out), ctypes.byref(nm))
    return nm.value, out[:len(k2)].copy()


def search_frames(info, kps2, desc2, Tcw2, kps1, desc1, mp1, pos1, window, kp2mp, score, nnratio=0.9):
    """ORBmatcher::SearchByProjection(F1, F2, window, ...) on the CPU oracle ->
    (nmatches, kp2mp, score)."""
    k2, d2 = np.ascontiguousarray(kps2, KEYPOINT_DTYPE), np.ascontiguousarray(desc2, np.uint8)
    k1, d1 = np.ascontiguousarray(kps1, KEYPOINT_DTYPE), np.ascontiguousarray(desc1, np.uint8)
    m1, p1 = np.ascontiguousarray(mp1, np.int32), np.ascontiguousarray(pos1, np.float32)
    T = np.ascontiguousarray(Tcw2, np.float32).reshape(16)
    km, sc = np.array(kp2mp, np.int32), np.array(score, np.int32)
    nm = ctypes.c_int()
    o = orc()
    o.orc_search_frames(ctypes.byref(info), _p(k2), _p(d2), len(k2), _p(T), _p(k1), _p(d1), _p(m1), _p(p1), len(k1),
                        window, ctypes.c_float(nnratio), _p(km), _p(sc), ctypes.byref(nm))
    return nm.value, km, sc


def search_kf_projection(info, kps, desc, Tcw, kf_kps, kf_mp, mps, mp_desc, found, th, orb_dist, kp2mp, score,
                         check_ori=True):
    """ORBmatcher::SearchByProjection(F, KF, sAlreadyFound, th, ORBdist) on the
    CPU oracle -> (nmatches, kp2mp, score)."""
    k, d = np.ascontiguousarray(kps, KEYPOINT_DTYPE), np.ascontiguousarray(desc, np.uint8)
    kk, km_ = np.ascontiguousarray(kf_kps, KEYPOINT_DTYPE), np.ascontiguousarray(kf_mp, np.int32)
    m, md = np.ascontiguousarray(mps), np.ascontiguousarray(mp_desc, np.uint8)
    f = np.ascontiguousarray(found, np.uint8)
    T = np.ascontiguousarray(Tcw, np.float32).reshape(16)
    km, sc = np.array(kp2mp, np.int32), np.array(score, np.int32)
    nm = ctypes.c_int()
    o = orc()
    o.orc_search_kf_projection(ctypes.byref(info), _p(k), _p(d), len(k), _p(T), _p(kk), _p(km_), len(kk), _p(m),
                               _p(md), _p(f), ctypes.c_float(th), orb_dist, int(check_ori), _p(km), _p(sc),
                               ctypes.byref(nm))
    return nm.value, km, sc


def reloc_candidates(words, values, db, kf_bad, cov_off, cov, query, state):
    """KeyFrameDatabase::DetectRelocalisationCandidates on the CPU oracle; db a
    pipeline.KeyframeDB, state a RELOC_KF_DTYPE array (updated in place) ->
    candidates."""
    w, v = np.ascontiguousarray(words, np.int32), np.ascontiguousarray(values, np.float64)
    nkf = db.nkf
    rq = np.ascontiguousarray(state["query"][:nkf], np.uint32)
    rw = np.ascontiguousarray(state["words"][:nkf], np.int32)
    rs = np.ascontiguousarray(state["score"][:nkf], np.float32)
    kb = np.ascontiguousarray(kf_bad if kf_bad is not None else np.zeros(nkf), np.uint8)
    co, cv = np.ascontiguousarray(cov_off, np.int32), np.ascontiguousarray(cov, np.int32)
    out = np.zeros(64, np.int32)
    nc = ctypes.c_int()
    o = orc()
    o.orc_reloc_candidates(_p(w), _p(v), len(w), nkf, _p(kb), _p(db.bow_off), _p(db.bow_words), _p(db.bow_values),
                           _p(co), _p(cv), ctypes.c_uint32(query), _p(rq), _p(rw), _p(rs), _p(out), ctypes.byref(nc))
    state["query"][:nkf], state["words"][:nkf], state["score"][:nkf] = rq, rw, rs
    return out[:nc.value].copy()
